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


def test_quirk_cases_run_on_oracle(oracle_lib):
    from _cases import u_quirks
    known, reads = u_quirks()
    hp = oracle_lib.haptag_reads(known, reads)
    assert set(np.unique(hp).tolist()) <= {0, 1, 254}
    # the cases reach every branch class: tagged both ways and undecided
    assert min(np.bincount(hp, minlength=255)[[0, 1, 254]]) > 20


@pytest.mark.gpu
@pytest.mark.parametrize("impl", ["wave", "thread"])
def test_haptag_quirks(oracle_lib, gpu_ctx, impl, monkeypatch):
    """Random MD strings ('^' runs spanning 64-char steps, '^' inside a run,
    leading letters / '^', long numbers), CIGARs of >64 ops with N/H/P, and
    2-3 known entries at one position; both kernels against the oracle."""
    from _cases import u_quirks
    if impl == "thread":
        monkeypatch.setenv("PF_K4_IMPL", "thread")
    for seed in (5, 6):
        known, reads = u_quirks(seed)
        ref = oracle_lib.haptag_reads(known, reads)
        out = gpu_ctx.haptag_reads(known, reads)
        assert np.array_equal(ref, out), (seed, np.argwhere(ref != out)[:5].ravel())
        name = "pf_k4_thread" if impl == "thread" else "pf_k4_haptag"
        assert name in gpu_ctx.kernel_times()


@pytest.mark.gpu
def test_haptag_contig_60x(oracle_lib, gpu_ctx):
    """One 4 Mb contig at 60x (20,000 reads of ~12 kb, SUP-like errors)."""
    known, reads, truth = make_u_batch(USpec(ref_len=4_000_000, n_reads=20000, mean_len=12000, seed=11))
    ref = oracle_lib.haptag_reads(known, reads)
    out = gpu_ctx.haptag_reads(known, reads)
    assert np.array_equal(ref, out), np.argwhere(ref != out)[:5].ravel()
    assert (out == truth).mean() > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize("md", [b"", b"12A3*4"])
def test_haptag_malformed_md(oracle_lib, gpu_ctx, md):
    """An empty or non-MD character fails the call (fatal in the reference,
    :1596 / :1621-1624); the read is left unphased."""
    from pomfret_amd._lib import PomfretError
    from pomfret_amd.abi import ReadAlnBatch
    known, reads, _ = make_u_batch(USpec(n_reads=20, seed=3))
    mds = [bytes(reads.md[reads.md_off[i]:reads.md_off[i + 1]]) for i in range(reads.n_reads)]
    mds[7] = md
    off = np.concatenate([[0], np.cumsum([len(m) for m in mds])])
    bad = ReadAlnBatch(start=reads.start, end=reads.end, cigar_off=reads.cigar_off, cigar=reads.cigar,
                       seq_off=reads.seq_off, seq_len=reads.seq_len, seq=reads.seq, md_off=off,
                       md=np.frombuffer(b"".join(mds), np.uint8))
    with pytest.raises(PomfretError):
        gpu_ctx.haptag_reads(known, bad)
