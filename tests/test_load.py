"""CPU tests of the window loader's oracle (a3/a4: read filters and 5mC call
extraction, blockjoin.c:1043-1173, 794-908, 605-792) and of the record-level
synthetic generator.  The hand-made records carry expected calls worked out
from the reference's loops (tests/_aln_cases.py)."""
import numpy as np
import pytest

from tests._aln_cases import HANDMADE, LOAD_CFG_SMALL, handmade_batch, records_batch, synth_aln

NONE = 0xFFFFFFFF


def _calls(b, r):
    co = b.read_call_off
    return list(zip(b.call_pos[co[r]:co[r + 1]].tolist(), b.call_cat[co[r]:co[r + 1]].tolist()))


def test_handmade_records(oracle_lib):
    b, rec_read = oracle_lib.load_reads(LOAD_CFG_SMALL, handmade_batch())
    for i, (name, rec, want) in enumerate(HANDMADE):
        if want is None:
            assert rec_read[i] == NONE, name
            continue
        assert rec_read[i] != NONE, name
        r = int(rec_read[i])
        assert _calls(b, r) == want, name
        assert b.read_start[r] == rec["pos"], name


def test_read_end_is_bam_endpos(oracle_lib):
    """bam_endpos: pos + M/D/N/=/X lengths of the whole CIGAR, also past the N
    that stops the call walk."""
    b, rec_read = oracle_lib.load_reads(LOAD_CFG_SMALL, handmade_batch())
    names = [h[0] for h in HANDMADE]
    r = int(rec_read[names.index("stop_at_n")])
    assert b.read_end[r] == 800 + 3 + 100 + 3
    r = int(rec_read[names.index("clip_ins_del")])
    assert b.read_end[r] == 1000 + 4 + 2 + 2 + 5


def test_fatal_cigar_operation(oracle_lib):
    """A hard clip (or =, X, P) reached by the walk is fatal in the reference
    (exit(1) at blockjoin.c:776-779): the oracle reports it as an error."""
    a = records_batch([(0, 10, [dict(seq="ACGTTCGA", cigar="6M2H", mm="C+m?,0,0;", ml=[200, 10], pos=100)])])
    with pytest.raises(RuntimeError):
        oracle_lib.load_reads(LOAD_CFG_SMALL, a)
    # not reached: the walk stops at the soft clip first
    a = records_batch([(0, 10, [dict(seq="ACGTTCGA", cigar="6M2S1H", mm="C+m?,0,0;", ml=[200, 10], pos=100)])])
    b, rr = oracle_lib.load_reads(LOAD_CFG_SMALL, a)
    assert rr[0] == 0


def test_quality_bands_are_uint8(oracle_lib):
    """lo/hi reach fill_read_meth_record_from_bam_line as uint8_t (799): hi=256
    wraps to 0, so no call is 'no-call' or 'unmethylated' above lo."""
    from pomfret_amd.abi import LoadConfig
    a = records_batch([(0, 10, [dict(seq="ACGTTCGA", cigar="8M", mm="C+m?,0,0;", ml=[120, 10], pos=100)])])
    b, _ = oracle_lib.load_reads(LoadConfig(min_mapq=10, min_len=6, qual_lo=100, qual_hi=256), a)
    assert _calls(b, 0) == [(101, 0), (105, 1)]


def test_clean_reads_call_every_covered_cpg(oracle_lib):
    """Without sequencing errors or clips, every decoded call is sorted, no read
    is in implicit mode, and reverse-strand calls land on the CpG's C like the
    forward ones (the same site set from both strands)."""
    a = synth_aln(2, 30, 7, sub_rate=0.0, indel_rate=0.0, clip_frac=0.0, filt_frac=0.0)
    b, rr = oracle_lib.load_reads(LOAD_CFG_SMALL, a)
    co = b.read_call_off.astype(np.int64)
    recs = np.flatnonzero(rr != NONE)
    fwd_sites, rev_sites = set(), set()
    for rec in recs:
        r = int(rr[rec])
        p = b.call_pos[co[r]:co[r + 1]]
        assert np.all(np.diff(p.astype(np.int64)) > 0)
        (rev_sites if a.flag[rec] & 16 else fwd_sites).update(p.tolist())
    common = fwd_sites & rev_sites
    assert len(common) > 0.8 * min(len(fwd_sites), len(rev_sites))


def test_record_level_path_recovers_orientation(oracle_lib):
    """End to end on the oracle: records -> loader -> methphase recovers the
    planted cis/trans orientation of every window at 30x."""
    from pomfret_amd import Config
    a = synth_aln(4, 30, 11)
    b, _ = oracle_lib.load_reads(LOAD_CFG_SMALL, a)
    res = oracle_lib.methphase(Config.from_coverage(30, given=False), b, n_threads=4)
    assert np.array_equal(res.decision, a.meta["orient"])


def test_threaded_record_level_path_matches_two_step(oracle_lib):
    """orc_methphase_aln (per-window load + worker, threaded: the CPU
    baseline of the record-level bench) equals load_reads + methphase."""
    from pomfret_amd import Config, LoadConfig
    cfg = Config.from_coverage(30, given=False)
    a = synth_aln(3, 30, 12, clip_frac=0.5, filt_frac=0.1)
    b, _ = oracle_lib.load_reads(LoadConfig(), a)
    ref = oracle_lib.methphase(cfg, b, n_threads=2)
    got = oracle_lib.methphase_aln(cfg, LoadConfig(), a, n_threads=3)
    for f in ("decision", "dir_table", "dir_join", "dir_which_way", "win_n_sites", "win_n_reads"):
        assert np.array_equal(getattr(ref, f), getattr(got, f)), f
