"""Full-size parity pinned by committed SHA-256 digests (tests/golden/digests.json).

The digests were produced by the CPU oracle (tests/golden/make_digests.py) on
inputs drawn from the SplitMix64 uniform stream with fixed seeds.
  * test_oracle_reproduces_digests (CPU): the oracle still produces them.
  * test_hip_matches_digests (GPU): the HIP path, with the same inputs
    generated ON THE DEVICE by fhe_fill_uniform, produces the same bytes at
    the BASELINE.json configs C1-C4 and the metric config.
"""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from full_size_cases import CASES, SEED_A, SEED_B, SEED_KEY, digest, shapes  # noqa: E402

DIGESTS = json.load(open(os.path.join(HERE, "golden", "digests.json")))


def test_digest_file_covers_every_case():
    assert sorted(DIGESTS) == sorted(CASES)


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_digests(name):
    from make_digests import oracle_output

    o, y = oracle_output(name)
    assert [int(q) for q in o.moduli] == DIGESTS[name]["moduli"]
    assert digest(y) == DIGESTS[name]["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_hip_matches_digests(name):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import herdsman_amd.backend as hb

    hb.load_library()
    scheme, log_n, L, K, dnum, t, op, n_ct, extra = CASES[name]
    c = hb.Context(scheme, log_n, L, K, dnum, t=t, bfv_mult="hps" if extra == "hps" else "behz")
    assert [int(q) for q in c.moduli] == DIGESTS[name]["moduli"]
    sh = shapes(CASES[name])
    a = c.fill_uniform(hb.empty(sh["a"]), seed=SEED_A)
    if op in ("ntt_fwd", "ntt_inv"):
        (c.ntt_fwd if op == "ntt_fwd" else c.ntt_inv)(a)
        y = a
    else:
        b = c.fill_uniform(hb.empty(sh["b"]), seed=SEED_B) if "b" in sh else None
        y = hb.empty(tuple(DIGESTS[name]["shape"]))
        if op == "add":
            c.add(a, b, y)
        else:
            key = c.fill_uniform(hb.empty((dnum, 2, L + K, 1 << log_n)), seed=SEED_KEY)
            if op == "mul_relin":
                c.mul_relin(a, b, key, y)
            elif op == "rotate":
                c.rotate(a, c.galois_elt(extra), key, y)
            elif op == "keyswitch":
                c.keyswitch(a, key, y)
    torch.cuda.synchronize()
    assert digest(hb.to_host(y)) == DIGESTS[name]["sha256"]
    c.close()
