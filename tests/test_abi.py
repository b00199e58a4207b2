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
