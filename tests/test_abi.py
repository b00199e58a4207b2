"""CPU-side checks of the drop-in boundary (no GPU compute).

* libherdsman_fhe.so builds for gfx950, loads, and exports EVERY function the
  C ABI header include/plugins/fhe_backend.h declares;
* the Python binding's signature table covers the same set;
* without a GPU the backend refuses loudly (no CPU fallback).
"""
import os
import re
import subprocess

import pytest
import numpy as np

import herdsman_amd.backend as hb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "plugins", "fhe_backend.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fhe_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import herdsman_amd.backend as hb
    if not os.path.exists(hb.library_path()):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "herdsman_amd")], check=True)
    return hb.load_library()


def test_header_declares_the_operator_surface():
    names = declared_functions()
    for op in ("fhe_ntt_fwd", "fhe_ntt_inv", "fhe_add", "fhe_mul_relin", "fhe_keyswitch", "fhe_rotate",
               "fhe_bcast_key", "fhe_base_conv", "fhe_reduce", "fhe_reduce_ranks"):
        assert op in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    import herdsman_amd.backend as hb
    assert sorted(hb.SIGNATURES) == declared_functions()


def test_exports_via_nm():
    import herdsman_amd.backend as hb
    out = subprocess.run(["nm", "-D", "--defined-only", hb.library_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (fhe_[a-z0-9_]+)", out))
    assert set(declared_functions()) <= exported


def test_gfx950_code_object_present():
    import herdsman_amd.backend as hb
    data = open(hb.library_path(), "rb").read()
    assert b"gfx950" in data


def test_no_gpu_means_loud_failure(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import herdsman_amd.backend as hb
    with pytest.raises(hb.FheBackendError):
        hb.Context(hb.SCHEME_CKKS, 12, 2)


def test_reduce_schedule_c_matches_python(lib):
    """fhe_reduce_schedule (host-only ABI function; the tree fhe_reduce_ranks runs
    with RCCL) equals herdsman_amd.dist.reduce_schedule (the gloo-tested tree)."""
    import herdsman_amd.backend as hb
    from herdsman_amd.dist import reduce_schedule
    for world in range(1, 17):
        for root in range(world):
            for rank in range(world):
                assert hb.reduce_schedule(rank, world, root) == reduce_schedule(rank, world, root)
    with pytest.raises(hb.FheBackendError):
        hb.reduce_schedule(2, 2, 0)


def _bare_context(hb, log_n=12, L=3, K=2, dnum=2):
    """A Context with its parameters but no device handle: the argument checks
    run before anything crosses the ABI, so they are testable without a GPU."""
    c = hb.Context.__new__(hb.Context)
    c.lib, c.h = None, None
    c.scheme, c.log_n, c.n, c.L, c.K, c.dnum = 0, log_n, 1 << log_n, L, K, dnum
    c.moduli = np.zeros(L + K, dtype=np.uint64)
    c.device = 0
    return c


def test_binding_rejects_bad_shapes_and_devices():
    """a short output, a wrong key or a tensor on another device must be
    rejected in the binding, never handed to the kernels as a raw pointer."""
    import torch
    import herdsman_amd.backend as hb

    c = _bare_context(hb)
    ct = lambda n: torch.empty((n, 2, 3, 1 << 12), dtype=torch.int64)
    key = torch.empty((2, 2, 5, 1 << 12), dtype=torch.int64)
    bad = [
        lambda: c.mul_relin(ct(2), ct(2), key, ct(1)),                      # short output
        lambda: c.mul_relin(ct(2), ct(3), key, ct(2)),                      # operand batch mismatch
        lambda: c.mul_relin(ct(2), ct(2), key[:1], ct(2)),                  # wrong key
        lambda: c.rotate(ct(2), 5, torch.empty((2, 2, 3, 1 << 12), dtype=torch.int64), ct(2)),
        lambda: c.add(ct(1), ct(1), torch.empty((1, 2, 3, 1 << 11), dtype=torch.int64)),
        lambda: c.keyswitch(torch.empty((2, 2, 1 << 12), dtype=torch.int64), key, ct(2)),
        lambda: c.ntt_fwd(torch.empty((1, 3, 1 << 12), dtype=torch.int64), mod_begin=3),  # limbs past the moduli
        lambda: c.reduce(ct(3), hb.REDUCE_ADD, out=torch.empty((2, 3, 1 << 12), dtype=torch.int64)),
        lambda: c.mul_relin(ct(2), ct(2), key, ct(2)),                      # right shapes, host tensors
    ]
    for i, f in enumerate(bad):
        with pytest.raises(hb.FheBackendError):
            f()


def test_build_id_ties_library_to_sources(lib, tmp_path):
    """the library carries the hash of the sources it was
    built from; the Makefile, the library and backend.source_build_id agree,
    and a mutated source tree makes the loader refuse the library."""
    import shutil
    import subprocess

    made = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "herdsman_amd"), "build-id"],
                          check=True, capture_output=True, text=True).stdout.strip()
    assert hb.check_build_id(lib) == made == hb.source_build_id()
    # a copy of the source tree with one kernel file changed
    pkg = tmp_path / "herdsman_amd"
    shutil.copytree(os.path.join(ROOT, "herdsman_amd", "csrc"), pkg / "csrc")
    (tmp_path / "include" / "plugins").mkdir(parents=True)
    shutil.copy(os.path.join(ROOT, "include", "plugins", "fhe_backend.h"), tmp_path / "include" / "plugins")
    assert hb.source_build_id(str(pkg)) == made
    with open(pkg / "csrc" / "ntt.hip", "a") as f:
        f.write("// edited after the build\n")
    assert hb.source_build_id(str(pkg)) != made
    with pytest.raises(hb.FheBackendError, match="built from other sources"):
        hb.check_build_id(lib, str(pkg))
