"""CPU tests of the oracle (test infrastructure) against the reference's own
fixtures, hand-worked cases of the reference algorithm and an independent
Fisher implementation.  No GPU needed.

Parity pinning (see DESIGN.md "Oracle"):
  * window definition (VCF PS -> gaps, merge_close_intervals) is pinned by the
    reference's example fixture tests/golden/example/ (copied data files);
  * Fisher's exact test is pinned against scipy.stats.fisher_exact;
  * the methylation core is "parity unpinned": the reference cannot be built in
    this image (htslib absent) and ships no vectors for it (example/phased.bam
    is missing); the hand-worked cases below follow the reference source line
    by line (blockjoin.c:3357-3451 for get_mmr_of_read).
"""
import gzip
import os

import numpy as np
import pytest

from pomfret_amd.abi import Config, WindowBatch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# --------------------------------------------------------------------------
# reference example fixture: window definition (f3 row)
def test_example_vcf_gaps(oracle_lib):
    """example/variants.vcf.gz: PS 9599993 block then PS 11147866 block; the
    single unphased gap is [last POS of block 1, PS of block 2] (blockjoin.c:1416-1418)."""
    res = oracle_lib.vcf_gaps(os.path.join(GOLD, "example", "variants.vcf.gz"))
    assert len(res) == 1
    c = res[0]
    assert c["name"] == "chr6"
    assert c["abs_start"] == 11082691
    assert c["abs_end"] == 11154381
    assert c["raw"] == [(11092382, 11147866)]
    assert c["gaps"] == [(11092382, 11147866)]
    assert c["dropped"] == []


def test_example_golden_outputs_semantics():
    """The golden outputs (older reference build) record
    one TRANS join of that gap: one merged GTF block whose ID is the block start,
    and the second block's phased GTs flipped under PS 11082691."""
    gtf = open(os.path.join(GOLD, "example", "output.mp.gtf")).read().split("\t")
    assert gtf[0] == "chr6" and gtf[3] == "11082691" and gtf[4].startswith("11154381")
    vin = {}
    with gzip.open(os.path.join(GOLD, "example", "variants.vcf.gz"), "rt") as f:
        for line in f:
            if line[0] != "#":
                t = line.rstrip("\n").split("\t")
                vin[int(t[1])] = t[9].split(":")[0]
    flipped = []
    with open(os.path.join(GOLD, "example", "output.mp.vcf")) as f:
        for line in f:
            if line[0] == "#":
                continue
            t = line.rstrip("\n").split("\t")
            gt = t[9].split(":")[0]
            pos = int(t[1])
            if gt != vin[pos]:
                flipped.append(pos)
                assert gt == vin[pos][::-1]       # a|b -> b|a : trans (decision 1)
                assert t[9].split(":")[-1] == "11082691"
    assert flipped[:2] == [11147866, 11153400]


# --------------------------------------------------------------------------
# search_arr (blockjoin.c:339-421)
@pytest.mark.parametrize("arr", [[5, 7, 7, 7, 9], list(range(0, 200, 2)) + [200, 200, 200]])
def test_search_arr(oracle_lib, arr):
    a = np.array(arr, np.uint32)
    assert oracle_lib.search_arr(a, a[0] - 1 if a[0] else 0, 0)[0] in (-1, 1)
    assert oracle_lib.search_arr(a, a[-1] + 1, 0) == (-2, 0xFFFFFFFF)
    for v in sorted(set(arr)):
        st, i = oracle_lib.search_arr(a, v, 0)
        assert st == 1 and i == arr.index(v)                     # leftmost hit
        st, i = oracle_lib.search_arr(a, v, 1)
        assert st == 1 and i == len(arr) - 1 - arr[::-1].index(v)  # rightmost hit
    st, i = oracle_lib.search_arr(a, arr[0] + 1, 0)
    if arr[0] + 1 not in arr:
        assert st == 0 and a[i] > arr[0] + 1 and (i == 0 or a[i - 1] < arr[0] + 1)
    assert oracle_lib.search_arr(np.zeros(0, np.uint32), 3, 0)[0] == -3


# --------------------------------------------------------------------------
# Fisher: htslib kt_fisher_exact restatement vs scipy (independent implementation)
@pytest.mark.parametrize("t", [(0, 13, 15, 0), (28, 0, 0, 20), (3, 1, 1, 3), (10, 2, 3, 15),
                               (5, 5, 5, 5), (0, 0, 0, 0), (1, 0, 0, 0), (40, 3, 2, 35),
                               (100, 1, 0, 120), (12, 5, 4, 11)])
def test_fisher_vs_scipy(oracle_lib, t):
    scipy_stats = pytest.importorskip("scipy.stats")
    _, left, right, two = oracle_lib.fisher(*t)
    if sum(t) == 0 or min(t[0] + t[1], t[2] + t[3], t[0] + t[2], t[1] + t[3]) == 0:
        assert two == 1.0
        return
    ref = scipy_stats.fisher_exact([[t[0], t[1]], [t[2], t[3]]], alternative="two-sided").pvalue
    assert two == pytest.approx(ref, rel=1e-6, abs=1e-300)
    lref = scipy_stats.fisher_exact([[t[0], t[1]], [t[2], t[3]]], alternative="less").pvalue
    assert left == pytest.approx(lref, rel=1e-6, abs=1e-300)


def test_fisher_product_matches_oracle(oracle_lib):
    """pf_fisher_exact (product host epilogue) == oracle restatement, bit for bit."""
    from pomfret_amd import fisher_exact
    rng = np.random.default_rng(7)
    for _ in range(300):
        t = [int(x) for x in rng.integers(0, 60, 4)]
        assert fisher_exact(*t) == oracle_lib.fisher(*t)


# --------------------------------------------------------------------------
# hand-worked methmer cases (get_mmr_of_read, blockjoin.c:3357-3451)
def _handmade_window():
    """Sites 100,200,300,400 carried by reads A and B; 30 left-side tagged reads
    with calls only at 50 (never a site) satisfy the left-coverage check."""
    reads = []
    for i in range(30):
        reads.append((10, 60, i % 2, [(50, 0)]))
    reads.append((90, 500, 254, [(100, 0), (200, 1), (300, 0), (400, 1)]))   # A: m u m u
    reads.append((90, 500, 254, [(100, 1), (200, 0), (300, 1), (400, 0)]))   # B: u m u m
    off = np.cumsum([0] + [len(r[3]) for r in reads])
    return WindowBatch(
        win_start=[60], win_end=[70], win_read_off=[0, len(reads)],
        read_start=[r[0] for r in reads], read_end=[r[1] for r in reads],
        read_hp=[r[2] for r in reads], read_call_off=off,
        call_pos=[c[0] for r in reads for c in r[3]], call_cat=[c[1] for r in reads for c in r[3]])


def test_methmers_forward_handworked(oracle_lib):
    cfg = Config(k=3, k_span=5000, cov_for_selection=1, cov_for_runtime=2, n_cand=4)
    b = _handmade_window()
    real, starts, lens = oracle_lib.window_sites(cfg, b, 0, 0)
    assert real.tolist() == [100, 200, 300, 400]
    assert starts.tolist() == [100, 200, 300, 400]
    assert lens.tolist() == [3, 2, 1, 1]               # j=min(i+k,n-1); len=j-i, 1 if j==i
    n, st, keys = oracle_lib.window_methmers(cfg, b, 0, 0)
    assert n[:30].tolist() == [0] * 30
    # A: entries at sites 0..2 (last call 400 is an exact hit -> exclusive):
    #   "mum"=0b000100=4, "um"=4, "m"=0 ; B: "umu"=17, "mu"=1, "u"=1
    assert n[30:].tolist() == [3, 3] and st[30:].tolist() == [0, 0]
    assert keys.tolist() == [4, 4, 0, 17, 1, 1]


def test_methmers_backward_duplicate_start_quirk(oracle_lib):
    """Direction 1: every site's methmer starts at site 0, so sites_starts =
    [100,100,100,100]; indices 0 AND 1 both enter the merge buffer (the `i>1`
    test, blockjoin.c:3391), giving entry 0 the character '-' (2)."""
    cfg = Config(k=3, k_span=5000, cov_for_selection=1, cov_for_runtime=2, n_cand=4)
    b = _handmade_window()
    real, starts, lens = oracle_lib.window_sites(cfg, b, 0, 1)
    assert starts.tolist() == [100, 100, 100, 100]
    assert lens.tolist() == [1, 1, 2, 3]
    n, st, keys = oracle_lib.window_methmers(cfg, b, 0, 1)
    # A: from entry(idx0): j=0 "-"=2, j=1 "-"=2, j=2 "-m"=8, j=3 incomplete;
    #    from entry(idx1): j=1 "m"=0, j=2/j=3 incomplete
    # B: same with 'u' (1): 2, 2, "-u"=9, then "u"=1
    assert n[30:].tolist() == [4, 4] and st[30:].tolist() == [0, 0]
    assert keys.tolist() == [2, 2, 8, 0, 2, 2, 9, 1]


def test_methmers_span_limit(oracle_lib):
    """k_span smaller than the site spacing: every methmer has length 1."""
    cfg = Config(k=3, k_span=50, cov_for_selection=1, cov_for_runtime=2, n_cand=4)
    b = _handmade_window()
    _, _, lens0 = oracle_lib.window_sites(cfg, b, 0, 0)
    _, _, lens1 = oracle_lib.window_sites(cfg, b, 0, 1)
    assert lens0.tolist() == [1, 1, 1, 1] and lens1.tolist() == [1, 1, 1, 1]


def test_left_coverage_check(oracle_lib):
    """Fewer than 15 left-side reads of a haplotype -> rs->n = 0, window skipped
    (blockjoin.c:1161-1163); decision stays -1 and tags are returned untouched."""
    b = _handmade_window()
    b.read_hp[:30] = 0                      # no hp1 reads on the left
    cfg = Config(k=3, k_span=5000, cov_for_selection=1, cov_for_runtime=2, n_cand=4)
    res = oracle_lib.methphase(cfg, b)
    assert res.decision.tolist() == [-1]
    assert res.win_n_sites.tolist() == [0] and res.win_n_reads.tolist() == [0]
    assert np.array_equal(res.read_hp, b.read_hp)


def test_synth_truth_recovered(oracle_lib):
    """On clean synthetic pileups the oracle recovers the simulated cis/trans
    orientation of (almost) every window (sanity of the restatement)."""
    from pomfret_amd.synth import SynthSpec, make_batch
    b = make_batch(SynthSpec(n_windows=12, coverage=30, seed=5))
    res = oracle_lib.methphase(Config.from_coverage(30, given=False), b, n_threads=4)
    joined = res.decision >= 0
    assert joined.sum() >= 10
    assert np.array_equal(res.decision[joined], b.meta["orient"][joined])


def test_golden_synth_vectors(oracle_lib):
    """Regression pin of the oracle on committed synthetic vectors
    (tests/golden/make_synth_golden.py)."""
    from pomfret_amd.synth import SynthSpec, make_batch
    g = np.load(os.path.join(GOLD, "synth_oracle.npz"), allow_pickle=False)
    for tag in ("c30", "c60", "mix"):
        dflt = SynthSpec()
        spec = SynthSpec(**{k: type(getattr(dflt, k))(v) for k, v in
                            zip(g[f"{tag}_spec_keys"].tolist(), g[f"{tag}_spec_vals"].tolist())})
        b = make_batch(spec)
        cfg = Config(*g[f"{tag}_cfg"].tolist())
        res = oracle_lib.methphase(cfg, b, n_threads=4)
        assert np.array_equal(res.decision, g[f"{tag}_decision"])
        assert np.array_equal(res.dir_table, g[f"{tag}_table"])
        assert np.array_equal(res.win_n_sites, g[f"{tag}_sites"])
        assert np.array_equal(res.read_hp, g[f"{tag}_hp"])


def test_t8_site_counter_wrap(oracle_lib):
    """T8: a site's meth/unmeth counts wrap at 4096 (u16 counters, 12-bit
    count, blockjoin.c:3210-3238); the sites of tests/_cases.t8_counter_wrap
    worked out by hand."""
    from tests._cases import T8_CFG, T8_SITES, t8_counter_wrap
    b = t8_counter_wrap()
    for d in (0, 1):
        real, _, _ = oracle_lib.window_sites(T8_CFG, b, 0, d)
        assert real.tolist() == T8_SITES          # dir 1 is reversed back after its ranges (3307-3329)
    assert oracle_lib.methphase(T8_CFG, b).win_n_sites.tolist() == [len(T8_SITES)]


def test_t6_range_index_wrap(oracle_lib):
    """T6: with every site right of e, direction 1's mmr_min_i wraps to
    UINT32_MAX (blockjoin.c:3999-4003) and no read is ever tagged in that
    direction; direction 0 tags reads (tests/_cases.t6_range_wrap)."""
    from tests._cases import t6_range_wrap
    cfg = Config(k=3, k_span=5000, cov_for_selection=4, cov_for_runtime=8, n_cand=8)
    b = t6_range_wrap()
    ids, tags, scores, counts = oracle_lib.trace(cfg, b)
    assert counts[0, 1] == 0 and counts[0, 0] > 0
    res = oracle_lib.methphase(cfg, b)
    assert res.dir_join[0, 1] == -1 and res.decision[0] == -1
