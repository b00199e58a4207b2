"""The IWorkerGroup adaptor (herdsman_amd/host/gpu_worker_group.cpp) driven the
way herdsman's Executor drives a worker group (schedule_task, then
set_completion_callback; /root/reference/src/execution/executor/executor.cpp:82-94).

CPU tests: the completion hand-off never loses a task even when the task
finishes before the callback is attached, and a task on a machine without a
GPU fails loudly (Status::ERROR), never on a CPU fallback.
GPU tests: MapTask / ReduceTask end to end over herdsman's partition-file
layout (<storage>/<session>/<frame>/<partition>, rows = u32 length + payload,
storage_service.cpp:19-28,233-240) and key-file layout
(<key_dir>/<session>/<schema>.key, key_service.cpp:28-31), bit-exact vs the
CPU oracle.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WG_RUN = os.path.join(ROOT, "herdsman_amd", "bin", "wg_run")


@pytest.fixture(scope="module")
def wg_run():
    if not os.path.exists(WG_RUN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "herdsman_amd"), "host"], check=True)
    return WG_RUN


# ------------------------------------------------------------- formats
def fnv(moduli):
    h = 0xcbf29ce484222325
    for q in moduli:
        for b in range(8):
            h ^= (int(q) >> (8 * b)) & 0xff
            h = (h * 0x100000001b3) & (2**64 - 1)
    return h


def ct_row(o, cts):
    """row payload: concatenated (CtHeader + words) ciphertexts, each at its own
    level (its limb count, CKKS)."""
    out = b""
    for ct in cts:
        lvl = ct.shape[-2]
        hdr = struct.pack("<IHBBIIQ", 0x54434648, 1, o.scheme, 1 if o.scheme == 0 else 0, o.log_n, lvl,
                          fnv(o.moduli[:lvl]))
        out += hdr + np.ascontiguousarray(ct, dtype=np.uint64).tobytes()
    return out


def parse_row(o, payload, level=None):
    assert struct.unpack_from("<I", payload)[0] == 0x54434648
    lvl = struct.unpack_from("<I", payload, 12)[0]
    assert lvl == (o.L if level is None else level)
    assert struct.unpack_from("<Q", payload, 16)[0] == fnv(o.moduli[:lvl])
    return np.frombuffer(payload[24:], dtype=np.uint64).reshape(2, lvl, o.n)


def write_partition(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        for r in rows:
            f.write(struct.pack("<I", len(r)) + r)


def read_partition(path):
    data, rows, off = open(path, "rb").read(), [], 0
    while off < len(data):
        (n,) = struct.unpack_from("<I", data, off)
        rows.append(data[off + 4:off + 4 + n])
        off += 4 + n
    return rows


def write_keys(path, o, relin, galois):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        f.write(struct.pack("<IHBBIIIIIIQ", 0x424B4648, 1, o.scheme, 0, o.log_n, o.L, o.K, o.dnum,
                            1 + len(galois), 0, fnv(o.moduli[:o.L + o.K])))
        f.write(struct.pack("<II", 0, 0) + np.ascontiguousarray(relin).tobytes())
        for g, k in galois.items():
            f.write(struct.pack("<II", 1, g) + np.ascontiguousarray(k).tobytes())


def params_arg(o, tmp):
    mf = os.path.join(tmp, "moduli.txt")
    with open(mf, "w") as f:
        f.write("\n".join(str(int(q)) for q in o.moduli))
    return f"{o.scheme},{o.log_n},{o.L},{o.K},{o.dnum},{o.t},{mf}"


# ---------------------------------------------------------------- CPU
def test_completion_handoff_never_loses_a_task(wg_run):
    r = subprocess.run([wg_run, "race", "200"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "200/200 delivered" in r.stdout


def test_no_gpu_task_fails_loudly(wg_run, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([wg_run, "map", str(tmp_path), str(tmp_path), "s", "0", "0,12,2,1,1,0", "in", "0", "out",
                        "in0", "in0", "add"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "status: ERROR" in r.stdout


# host sanitizers (ASan + UBSan on the adaptor; the HIP library is not instrumented)
SAN_ENV = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def wg_run_san():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "herdsman_amd"), "sanitize"], check=True)
    return os.path.join(ROOT, "herdsman_amd", "bin", "wg_run_san")


def _clean(r):
    out = r.stdout + r.stderr
    return "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out


def test_sanitized_completion_handoff(wg_run_san):
    r = subprocess.run([wg_run_san, "race", "200"], capture_output=True, text=True, timeout=300, env=SAN_ENV)
    assert r.returncode == 0 and _clean(r), r.stdout + r.stderr
    assert "200/200 delivered" in r.stdout


def test_sanitized_no_gpu_task(wg_run_san, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([wg_run_san, "map", str(tmp_path), str(tmp_path), "s", "0", "0,12,2,1,1,0", "in", "0", "out",
                        "in0", "in0", "add"], capture_output=True, text=True, timeout=120, env=SAN_ENV)
    assert r.returncode == 2 and "status: ERROR" in r.stdout and _clean(r), r.stdout + r.stderr


# ---------------------------------------------------------------- GPU
def _setup(tmp_path, scheme, log_n, L, K, dnum, t=0):
    from oracle_ffi import Oracle
    o = Oracle(scheme, log_n, L, K, dnum, t=t)
    return o, str(tmp_path / "storage"), str(tmp_path / "keys")


@pytest.mark.gpu
def test_gpu_map_task_mul_rotate(wg_run, tmp_path):
    from oracle_ffi import SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 12, 4, 2, 2)
    rows = 5
    a = o.uniform((rows, 2, o.L, o.n), seed=1)
    b = o.uniform((rows, 2, o.L, o.n), seed=2)
    rlk = o.uniform(o.key_shape(), seed=3)
    g = o.galois_elt(3)
    gk = o.uniform(o.key_shape(), seed=4)
    write_partition(os.path.join(storage, "sess", "frameA", "2"), [ct_row(o, [a[i], b[i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sess", "7.key"), o, rlk, {g: gk})
    r = subprocess.run([wg_run, "map", storage, keys, "sess", "7", params_arg(o, str(tmp_path)), "frameA", "2",
                        "frameB", "in0", "in1", "mul", "rot:3"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.stack([parse_row(o, p) for p in read_partition(os.path.join(storage, "sess", "frameB", "2"))])
    want = o.rotate(o.mul_relin(a, b, rlk), g, gk)
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,steps,lvl", [(16, (0, 1, 3), 11), (12, (1, 2), 4),
                                             (12, (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10), 4)])
def test_gpu_map_task_rotsum_hoisted(wg_run, tmp_path, log_n, steps, lvl):
    """ROTSUM: the sum of the input's rotations by the given steps (0 = the input
    itself), double-hoisted (fhe_rotate_sum_hoisted_at: one ModUp, one ModDown);
    at N=2^16 on level-11 rows (the fused gather path at a reduced level), at
    N=2^12 after a product (the generic path)."""
    from oracle_ffi import SCHEME_CKKS
    L, K, dnum = (12, 4, 3) if log_n == 16 else (4, 2, 2)
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, log_n, L, K, dnum)
    rows = 2
    a = o.uniform((rows, 2, lvl, o.n), seed=61)
    b = o.uniform((rows, 2, lvl, o.n), seed=62)
    rlk = o.uniform(o.key_shape(), seed=63)
    rot = [k for k in steps if k]
    gs = [o.galois_elt(k) for k in rot]
    gks = [o.uniform(o.key_shape(), seed=70 + k) for k in rot]
    write_partition(os.path.join(storage, "sr", "fa", "0"), [ct_row(o, [a[i], b[i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sr", "0.key"), o, rlk, dict(zip(gs, gks)))
    prog = ["in0"] if log_n == 16 else ["in0", "in1", "mul"]
    r = subprocess.run([wg_run, "map", storage, keys, "sr", "0", params_arg(o, str(tmp_path)), "fa", "0", "fb"]
                       + prog + ["rotsum:" + ",".join(map(str, steps))], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.stack([parse_row(o, p, level=lvl) for p in read_partition(os.path.join(storage, "sr", "fb", "0"))])
    x = a if log_n == 16 else o.mul_relin_at(a, b, rlk, lvl)
    terms = [o.rotate_sum_hoisted(x, gs, np.stack(gks), lvl)] + ([x] if 0 in steps else [])
    qs = o.moduli[:lvl].astype(object)[None, None, :, None]
    want = sum(t.astype(object) for t in terms) % qs
    assert np.array_equal(got, want.astype(np.uint64))


@pytest.mark.gpu
def test_gpu_map_task_rotsum_bfv(wg_run, tmp_path):
    """ROTSUM on BFV rows (C3 parameters): the double-hoisted sum in coefficient form."""
    from oracle_ffi import SCHEME_BFV
    o, storage, keys = _setup(tmp_path, SCHEME_BFV, 15, 8, 4, 2, t=65537)
    rows = 2
    a = o.uniform((rows, 2, o.L, o.n), seed=81)
    rlk = o.uniform(o.key_shape(), seed=82)
    steps = (0, 2, 5)
    gs = [o.galois_elt(k) for k in steps if k]
    gks = [o.uniform(o.key_shape(), seed=83 + i) for i in range(len(gs))]
    write_partition(os.path.join(storage, "sb", "fa", "1"), [ct_row(o, [a[i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sb", "1.key"), o, rlk, dict(zip(gs, gks)))
    r = subprocess.run([wg_run, "map", storage, keys, "sb", "1", params_arg(o, str(tmp_path)), "fa", "1", "fb",
                        "in0", "rotsum:0,2,5"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.stack([parse_row(o, p) for p in read_partition(os.path.join(storage, "sb", "fb", "1"))])
    terms = [o.rotate_sum_hoisted(a, gs, np.stack(gks)), a]
    qs = o.moduli[:o.L].astype(object)[None, None, :, None]
    want = sum(t.astype(object) for t in terms) % qs
    assert np.array_equal(got, want.astype(np.uint64))


@pytest.mark.gpu
def test_gpu_map_task_ckks_levels(wg_run, tmp_path):
    """A depth-2 CKKS circuit through the worker group: rows carry ciphertexts at
    levels 12, 12 and 11; in0 in1 mul rescale in1 mul in2 add rescale runs the
    second product at level 11 (in1's 12th limb dropped), adds the level-11
    input and writes level-10 rows, bit-exact vs the oracle's level ops."""
    from oracle_ffi import SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 16, 12, 4, 3)
    rows = 2
    a = o.uniform((rows, 2, 12, o.n), seed=31)
    b = o.uniform((rows, 2, 12, o.n), seed=32)
    c = o.uniform((rows, 2, 11, o.n), seed=33)
    rlk = o.uniform(o.key_shape(), seed=34)
    write_partition(os.path.join(storage, "sl", "fa", "0"), [ct_row(o, [a[i], b[i], c[i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sl", "0.key"), o, rlk, {})
    r = subprocess.run([wg_run, "map", storage, keys, "sl", "0", params_arg(o, str(tmp_path)), "fa", "0", "fb",
                        "in0", "in1", "mul", "rescale", "in1", "mul", "in2", "add", "rescale"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.stack([parse_row(o, p, level=10) for p in read_partition(os.path.join(storage, "sl", "fb", "0"))])
    p1 = o.rescale(o.mul_relin_at(a, b, rlk, 12), 12)
    p2 = o.mul_relin_at(p1, np.ascontiguousarray(b[:, :, :11]), rlk, 11)
    qs = o.moduli[:11].astype(object)[None, None, :, None]
    p3 = ((p2.astype(object) + c) % qs).astype(np.uint64)
    assert np.array_equal(got, o.rescale(p3, 11))


@pytest.mark.gpu
def test_gpu_reduce_task_add_and_mul_trees(wg_run, tmp_path):
    from oracle_ffi import SCHEME_BFV
    o, storage, keys = _setup(tmp_path, SCHEME_BFV, 12, 3, 3, 1, t=65537)
    parts = {"p0": 3, "p1": 1, "p2": 3}
    cts, i = [], 0
    for name, cnt in parts.items():
        rows = []
        for _ in range(cnt):
            ct = o.uniform((1, 2, o.L, o.n), seed=100 + i)[0]
            cts.append(ct)
            rows.append(ct_row(o, [ct]))
            i += 1
        write_partition(os.path.join(storage, "s2", name, "0"), rows)
    rlk = o.uniform(o.key_shape(), seed=9)
    write_keys(os.path.join(keys, "s2", "1.key"), o, rlk, {})
    inputs = [f"{n}:0" for n in parts]
    args = [wg_run, "reduce", storage, keys, "s2", "1", params_arg(o, str(tmp_path))]
    r = subprocess.run(args + ["outA", "0"] + inputs, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = parse_row(o, read_partition(os.path.join(storage, "s2", "outA", "0"))[0])
    want = cts[0]
    for c in cts[1:]:
        want = o.ct_add(want[None], c[None])[0]
    assert np.array_equal(got, want)
    # multiplicative tree: replicate the group's level order exactly
    r = subprocess.run(args + ["outM", "0"] + inputs + ["--", "mul"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = parse_row(o, read_partition(os.path.join(storage, "s2", "outM", "0"))[0])
    live = [c for c in cts]
    while len(live) > 1:
        half = len(live) // 2
        lo = np.stack(live[:half])
        hi = np.stack(live[len(live) - half:])
        comb = o.mul_relin(lo, hi, rlk)
        live = list(comb) + live[half:len(live) - half]
    assert np.array_equal(got, live[0])


@pytest.mark.gpu
def test_gpu_reduce_task_chunked(wg_run, tmp_path):
    """Rows staged max_batch (here 2) at a time: each chunk is a balanced tree,
    the chunk results merge like a binary counter (older operand first).  CKKS
    at level 7 (the rows' own level), 7 rows over 3 partitions, one empty."""
    from oracle_ffi import SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 13, 8, 2, 3)
    lvl = 7
    parts = {"q0": 3, "q1": 0, "q2": 4}
    cts, i = [], 0
    for name, cnt in parts.items():
        rows = []
        for _ in range(cnt):
            ct = o.uniform((1, 2, lvl, o.n), seed=200 + i)[0]
            cts.append(ct)
            rows.append(ct_row(o, [ct]))
            i += 1
        write_partition(os.path.join(storage, "s3", name, "0"), rows)
    rlk = o.uniform(o.key_shape(), seed=29)
    write_keys(os.path.join(keys, "s3", "0.key"), o, rlk, {})
    env = dict(os.environ, WG_MAX_BATCH="2")
    args = [wg_run, "reduce", storage, keys, "s3", "0", params_arg(o, str(tmp_path)), "outM", "0"]
    r = subprocess.run(args + [f"{n}:0" for n in parts] + ["--", "mul"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    got = parse_row(o, read_partition(os.path.join(storage, "s3", "outM", "0"))[0], level=lvl)
    assert np.array_equal(got, _reduce_tree_chunked(o, cts, rlk, True, 2, lvl))


def _reduce_tree_chunked(o, cts, rlk, mul, chunk, lvl=None):
    """The worker group's ReduceTask tree: chunks of `chunk` rows in partition
    order, each a balanced tree (fhe_reduce_at), the chunk results merged like a
    binary counter (older operand first)."""
    lvl = o.L if lvl is None else lvl
    qs = o.moduli[:lvl].astype(object)[None, :, None]

    def op(x, y):
        if mul:  # BFV has no level views: the plain product
            return (o.mul_relin(x[None], y[None], rlk) if lvl == o.L else o.mul_relin_at(x[None], y[None], rlk, lvl))[0]
        return ((x.astype(object) + y) % qs).astype(np.uint64)

    def tree(items):
        live = list(items)
        while len(live) > 1:
            half = len(live) // 2
            comb = [op(live[j], live[len(live) - half + j]) for j in range(half)]
            live = comb + live[half:len(live) - half]
        return live[0]

    pend = []
    for c0 in range(0, len(cts), chunk):
        p, h = tree(cts[c0:c0 + chunk]), 0
        while pend and pend[-1][1] == h:
            p, h = op(pend.pop()[0], p), h + 1
        pend.append((p, h))
    while len(pend) > 1:
        p = pend.pop()[0]
        pend[-1] = (op(pend[-1][0], p), pend[-1][1])
    return pend[0][0]


@pytest.mark.gpu
@pytest.mark.parametrize("mult", ["behz", "hps"])
def test_gpu_map_task_bfv(wg_run, tmp_path, mult):
    from oracle_ffi import Oracle, SCHEME_BFV
    o, storage, keys = _setup(tmp_path, SCHEME_BFV, 13, 3, 2, 2, t=65537)
    if mult == "hps":
        o = Oracle(SCHEME_BFV, 13, 3, 2, 2, t=65537, bfv_mult="hps")
    rows = 3
    a = o.uniform((rows, 2, o.L, o.n), seed=21)
    b = o.uniform((rows, 2, o.L, o.n), seed=22)
    rlk = o.uniform(o.key_shape(), seed=23)
    write_partition(os.path.join(storage, "sb", "in", "0"), [ct_row(o, [a[i], b[i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sb", "1.key"), o, rlk, {})
    # (in0 * in1) + in0
    r = subprocess.run([wg_run, "map", storage, keys, "sb", "1", params_arg(o, str(tmp_path)) + "," + mult, "in",
                        "0", "out", "in0", "in1", "mul", "in0", "add"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.stack([parse_row(o, p) for p in read_partition(os.path.join(storage, "sb", "out", "0"))])
    assert np.array_equal(got, o.ct_add(o.mul_relin(a, b, rlk), a))


@pytest.mark.gpu
def test_gpu_bad_inputs_fail_the_task(wg_run, tmp_path):
    """A key file for other moduli, or a truncated ciphertext row, ends the task with
    Status::ERROR (no exception crosses the seam, nothing is written)."""
    from oracle_ffi import Oracle, SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 12, 3, 2, 2)
    other = Oracle(SCHEME_CKKS, 12, 3, 2, 2, moduli=np.concatenate([o.moduli[1:2], o.moduli[:1], o.moduli[2:]]))
    a = o.uniform((1, 2, o.L, o.n), seed=31)[0]
    write_partition(os.path.join(storage, "sx", "in", "0"), [ct_row(o, [a, a])])
    write_keys(os.path.join(keys, "sx", "0.key"), other, o.uniform(o.key_shape(), seed=32), {})
    base = [wg_run, "map", storage, keys, "sx", "0", params_arg(o, str(tmp_path)), "in", "0"]
    r = subprocess.run(base + ["out1", "in0", "in1", "mul"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 2 and "status: ERROR" in r.stdout, r.stdout + r.stderr
    assert not os.path.exists(os.path.join(storage, "sx", "out1", "0"))
    row = ct_row(o, [a, a])
    write_partition(os.path.join(storage, "sy", "in", "1"), [row[: len(row) - 8]])
    write_keys(os.path.join(keys, "sy", "0.key"), o, o.uniform(o.key_shape(), seed=33), {})
    r = subprocess.run([wg_run, "map", storage, keys, "sy", "0", params_arg(o, str(tmp_path)), "in", "1", "out2",
                        "in0", "in1", "mul"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 2 and "status: ERROR" in r.stdout, r.stdout + r.stderr
    assert not os.path.exists(os.path.join(storage, "sy", "out2", "1"))


@pytest.mark.gpu
def test_gpu_failed_batch_leaves_the_lane_usable(wg_run, tmp_path):
    """A bad row in a later batch of a task (one lane, one row per batch, so earlier
    batches are still in flight on the lane's stream when it is read) fails that task
    with Status::ERROR; the next task on the same lane reuses the staging buffers and
    is bit-exact (the catch path synchronises the lane before completing)."""
    from oracle_ffi import SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 12, 3, 2, 2)
    rows = 3
    a = o.uniform((rows, 2, o.L, o.n), seed=51)
    b = o.uniform((rows, 2, o.L, o.n), seed=52)
    rlk = o.uniform(o.key_shape(), seed=53)
    good = [ct_row(o, [a[i], b[i]]) for i in range(rows)]
    bad = bytearray(good[2])
    bad[0:4] = struct.pack("<I", 0xDEADBEEF)  # corrupt the CtHeader magic of the third row
    write_partition(os.path.join(storage, "sl", "in", "1"), good[:2] + [bytes(bad)])
    write_partition(os.path.join(storage, "sl", "in", "0"), good)
    write_keys(os.path.join(keys, "sl", "0.key"), o, rlk, {})
    env = dict(os.environ, WG_LANES="1", WG_MAX_BATCH="1")
    r = subprocess.run([wg_run, "map", storage, keys, "sl", "0", params_arg(o, str(tmp_path)), "in", "1,0", "out",
                        "in0", "in1", "mul"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 2, r.stdout + r.stderr
    assert r.stdout.split("status: ")[1:] == ["ERROR\n", "COMPLETED\n"], r.stdout + r.stderr
    assert not os.path.exists(os.path.join(storage, "sl", "out", "1"))
    got = np.stack([parse_row(o, p) for p in read_partition(os.path.join(storage, "sl", "out", "0"))])
    assert np.array_equal(got, o.mul_relin(a, b, rlk))


def _chain(wg_run, tmp_path, o, storage, keys, session, schema, parts, prog1, prog2, resident, write_behind):
    env = dict(os.environ, WG_MAX_BATCH="2", WG_LANES="3", WG_RESIDENT_BYTES=str(resident),
               WG_WRITE_BEHIND="1" if write_behind else "0")
    r = subprocess.run([wg_run, "chain", storage, keys, session, str(schema), params_arg(o, str(tmp_path)), "fa",
                        str(parts), "fm", "fo"] + prog1 + ["--"] + prog2,
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("chain:")][0].split()
    return {line[i]: int(line[i + 1]) for i in range(1, len(line), 2)}


@pytest.mark.gpu
@pytest.mark.parametrize("resident,write_behind", [(1 << 34, False), (1 << 34, True), (0, False),
                                                   (3 * 2 * 4 * 4096 * 8 * 2, True)])
def test_gpu_chained_map_stages_resident_frames(wg_run, tmp_path, resident, write_behind):
    """herdsman chains Map stages through intermediate frames that the next stage
    reads back (execution_service.cpp:525-543).  Stage 1 "in0 in1 mul rescale"
    writes frame fm; stage 2 "in0 in0 mul rot:1" reads it.  With resident frames
    stage 2 reads fm from HBM (no pread, no H2D; resident_rows counts them), with
    write-behind fm's and fo's files are committed by the flusher; with no budget
    everything goes through the files; with a budget of 1.57 MB (one 5-row
    level-3 frame is 0.98 MB) each new frame evicts the previous one, so some
    stage-2 tasks read their input from the file.  Both frames' files are
    bit-exact against the oracle in every mode."""
    from oracle_ffi import SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 12, 4, 2, 2)
    parts, rows = 3, 5
    a = o.uniform((parts, rows, 2, o.L, o.n), seed=91)
    b = o.uniform((parts, rows, 2, o.L, o.n), seed=92)
    rlk = o.uniform(o.key_shape(), seed=93)
    g = o.galois_elt(1)
    gk = o.uniform(o.key_shape(), seed=94)
    for p in range(parts):
        write_partition(os.path.join(storage, "sc", "fa", str(p)), [ct_row(o, [a[p, i], b[p, i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sc", "0.key"), o, rlk, {g: gk})
    st = _chain(wg_run, tmp_path, o, storage, keys, "sc", 0, parts, ["in0", "in1", "mul", "rescale"],
                ["in0", "in0", "mul", "rot:1"], resident, write_behind)
    for p in range(parts):
        mid = o.rescale(o.mul_relin(a[p], b[p], rlk), o.L)
        got_mid = np.stack([parse_row(o, r, level=o.L - 1) for r in read_partition(os.path.join(storage, "sc", "fm", str(p)))])
        assert np.array_equal(got_mid, mid), p
        fin = o.rotate_at(o.mul_relin_at(mid, mid, rlk, o.L - 1), g, gk, o.L - 1)
        got = np.stack([parse_row(o, r, level=o.L - 1) for r in read_partition(os.path.join(storage, "sc", "fo", str(p)))])
        assert np.array_equal(got, fin), p
    assert st["rows"] == 2 * parts * rows
    if resident >= 1 << 34:
        assert st["resident_rows"] == parts * rows  # every stage-2 row came from HBM
    elif resident == 0:
        assert st["resident_rows"] == 0
    else:
        assert 0 < st["resident_rows"] < parts * rows  # the evicted partition was read from its file
    if write_behind and resident >= 1 << 34:
        assert st["flushed_rows"] == 2 * parts * rows  # every output frame written behind
    elif write_behind:
        # an output whose reservation fails (bytes of outputs still in flight cannot
        # be evicted) is written by its lane; the rest by the flusher
        assert 0 < st["flushed_rows"] <= 2 * parts * rows
    else:
        assert st["flushed_rows"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mul", [False, True])
def test_gpu_map_then_reduce_reads_resident_frames(wg_run, tmp_path, mul):
    """A ReduceTask over a Map stage's output partitions reads them from HBM and
    builds the same tree (chunks of max_batch rows across partitions) as from
    files: bit-exact against the oracle's tree."""
    from oracle_ffi import SCHEME_BFV
    o, storage, keys = _setup(tmp_path, SCHEME_BFV, 12, 3, 3, 1, t=65537)
    parts, rows = 3, 3
    a = o.uniform((parts, rows, 2, o.L, o.n), seed=95)
    b = o.uniform((parts, rows, 2, o.L, o.n), seed=96)
    rlk = o.uniform(o.key_shape(), seed=97)
    for p in range(parts):
        write_partition(os.path.join(storage, "sd", "fa", str(p)), [ct_row(o, [a[p, i], b[p, i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sd", "1.key"), o, rlk, {})
    st = _chain(wg_run, tmp_path, o, storage, keys, "sd", 1, parts, ["in0", "in1", "add"],
                ["reduce"] + (["mul"] if mul else []), 1 << 34, False)
    assert st["resident_rows"] == parts * rows
    mids = [((a[p].astype(object) + b[p]) % o.moduli[:o.L].astype(object)[None, None, :, None]).astype(np.uint64)
            for p in range(parts)]
    flat = list(np.concatenate(mids))
    (got_row,) = read_partition(os.path.join(storage, "sd", "fo", "0"))
    got = parse_row(o, got_row)
    want = _reduce_tree_chunked(o, flat, rlk, mul, 2)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_write_behind_failure_fails_the_consumers(wg_run, tmp_path):
    """with write-behind a MapTask completes when its output is
    in HBM, so a flush that fails later must still reach the executor.  Stage 1
    writes fm over 3 partitions; fm/2 cannot be committed (a non-empty directory
    sits at its path, which no rename replaces, root or not).  After the flush,
    stage 2's first scheduled task reports the session's failure and the task
    reading fm/2 fails; the task reading fm/1 completes bit-exactly."""
    from oracle_ffi import SCHEME_CKKS
    o, storage, keys = _setup(tmp_path, SCHEME_CKKS, 12, 3, 1, 3)
    parts, rows = 3, 2
    a = o.uniform((parts, rows, 2, o.L, o.n), seed=101)
    b = o.uniform((parts, rows, 2, o.L, o.n), seed=102)
    rlk = o.uniform(o.key_shape(), seed=103)
    for p in range(parts):
        write_partition(os.path.join(storage, "sw", "fa", str(p)), [ct_row(o, [a[p, i], b[p, i]]) for i in range(rows)])
    write_keys(os.path.join(keys, "sw", "0.key"), o, rlk, {})
    blocker = os.path.join(storage, "sw", "fm", "2")
    os.makedirs(blocker)
    open(os.path.join(blocker, "keep"), "w").close()
    env = dict(os.environ, WG_MAX_BATCH="2", WG_LANES="2", WG_RESIDENT_BYTES=str(1 << 34), WG_WRITE_BEHIND="1",
               WG_FLUSH_BETWEEN="1")
    r = subprocess.run([wg_run, "chain", storage, keys, "sw", "0", params_arg(o, str(tmp_path)), "fa", str(parts),
                        "fm", "fo", "in0", "in1", "mul", "--", "in0", "in0", "mul"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dict(ln.split(":", 1) for ln in r.stdout.splitlines() if ":" in ln)
    assert lines["stage1_flush"].strip() == "ERROR", r.stdout
    st2 = lines["stage2"].split()
    assert st2 == ["ERROR", "COMPLETED", "ERROR"], r.stdout + r.stderr
    assert "session sw" in r.stderr and "never committed" in r.stderr, r.stderr
    mid = o.mul_relin(a[1], b[1], rlk)
    got = np.stack([parse_row(o, x) for x in read_partition(os.path.join(storage, "sw", "fo", "1"))])
    assert np.array_equal(got, o.mul_relin(mid, mid, rlk))
    assert not os.path.isfile(os.path.join(storage, "sw", "fo", "2"))
