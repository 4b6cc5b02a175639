"""The --bam-is-untagged pre-pass (reference blockjoin.c:1545-1898)."""
import numpy as np
import pytest

from pomfret_amd.abi import KnownVars
from pomfret_amd.synth_u import USpec, make_u_batch

SPECS = {
    "sup": USpec(n_reads=400, seed=11),
    "hac": USpec(n_reads=400, sub_err=0.02, indel_err=0.01, seed=12),
    "dense_indels": USpec(n_reads=200, var_every=300, indel_frac=0.5, seed=13),
}


def test_oracle_recovers_truth(oracle_lib):
    known, reads, hap = make_u_batch(SPECS["sup"])
    hp = oracle_lib.haptag_reads(known, reads)
    tagged = hp < 2
    assert tagged.mean() > 0.95
    assert np.array_equal(hp[tagged], hap[tagged])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SPECS))
def test_haptag_parity(oracle_lib, gpu_ctx, name):
    known, reads, _ = make_u_batch(SPECS[name])
    ref = oracle_lib.haptag_reads(known, reads)
    out = gpu_ctx.haptag_reads(known, reads)
    assert np.array_equal(ref, out), np.argwhere(ref != out)[:5]


@pytest.mark.gpu
def test_haptag_no_known_variants(gpu_ctx):
    _, reads, _ = make_u_batch(USpec(n_reads=20, seed=3))
    empty = KnownVars(pos=np.zeros(0), len=np.zeros(0), op=np.zeros(0), haptag=np.zeros(0),
                      char_off=np.zeros(1), chars=np.zeros(0, np.uint8))
    assert (gpu_ctx.haptag_reads(empty, reads) == 254).all()
