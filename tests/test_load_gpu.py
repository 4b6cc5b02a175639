"""GPU parity of kernel K0 (the window loader on the device) against the CPU
oracle, through the C ABI (pf_batch_upload_aln).

Integer outputs must be bit-identical: which records are kept, every read's
calls (sorted by (pos, cat), as the methmer kernels consume them), the first
and last call in get_mod_poss_on_ref's order, read starts/ends, and then the
whole methphase result of the record-level batch.
"""
import os

import numpy as np
import pytest

from pomfret_amd.abi import LoadConfig

from tests._aln_cases import HANDMADE, LOAD_CFG_SMALL, aln_cases, handmade_batch, mm_fuzz_batch, records_batch

pytestmark = pytest.mark.gpu

NONE = 0xFFFFFFFF
CASES = aln_cases()


def _oracle_view(oracle_lib, lcfg, aln):
    b, rec_read = oracle_lib.load_reads(lcfg, aln)
    co = b.read_call_off.astype(np.int64)
    first = np.array([b.call_pos[co[r]] if co[r + 1] > co[r] else 0 for r in range(b.n_reads)], np.uint32)
    last = np.array([b.call_pos[co[r + 1] - 1] if co[r + 1] > co[r] else 0 for r in range(b.n_reads)], np.uint32)
    pos, cat = b.call_pos.copy(), b.call_cat.copy()
    for r in range(b.n_reads):
        o = np.lexsort((cat[co[r]:co[r + 1]], pos[co[r]:co[r + 1]]))
        pos[co[r]:co[r + 1]] = pos[co[r]:co[r + 1]][o]
        cat[co[r]:co[r + 1]] = cat[co[r]:co[r + 1]][o]
    return b, rec_read, pos, cat, first, last


def _check_calls(oracle_lib, gpu_ctx, cfg, lcfg, aln, tag):
    b, rec_read, pos, cat, first, last = _oracle_view(oracle_lib, lcfg, aln)
    db = gpu_ctx.upload_aln(cfg, aln, lcfg)
    off, gpos, gcat, gfirst, glast = db.debug_calls()      # K0 sizes the batch on the device
    assert db.n_reads == b.n_reads, tag
    assert np.array_equal(db.read_recs(), np.flatnonzero(rec_read != NONE)), tag
    assert np.array_equal(off, b.read_call_off), tag
    bad = np.flatnonzero(gpos != pos)
    assert bad.size == 0, f"{tag}: call_pos differs at {bad[:5].tolist()}"
    assert np.array_equal(gcat, cat), f"{tag}: call_cat differs at {np.flatnonzero(gcat != cat)[:5].tolist()}"
    assert np.array_equal(gfirst, first), tag
    assert np.array_equal(glast, last), tag
    return db, b


def test_handmade_records(oracle_lib, gpu_ctx):
    """The hand-made records of tests/_aln_cases.HANDMADE: K0's calls equal
    the oracle's and, record by record, the calls worked out BY HAND from the
    reference's loops and the SAM MM/ML specification (not from the oracle),
    so a change to the oracle cannot move both sides together.  The
    duplex-style records (C+m with C-m, several C m entries) rest on htslib's
    base-mod semantics, which no reference fixture holds: parity unpinned
    beyond these hand-worked expectations."""
    from pomfret_amd import Config
    aln = handmade_batch()
    db, b = _check_calls(oracle_lib, gpu_ctx, Config(), LOAD_CFG_SMALL, aln, "handmade")
    kept = [h for h in HANDMADE if h[2] is not None]
    assert db.n_reads == len(kept)
    off, gpos, gcat, _, _ = db.debug_calls()
    for r, (name, rec, want) in enumerate(kept):
        got = list(zip(gpos[off[r]:off[r + 1]].tolist(), gcat[off[r]:off[r + 1]].tolist()))
        assert got == sorted(want), name
    c = db.load_counters()
    assert c["seq_path"] >= 2 and c["implicit"] >= 2 and c["bad_mm"] >= 2
    # the duplex-style records (several C m entries) went through pf_k0_multi
    n_multi = sum(1 for h in HANDMADE if h[1].get("mm", "").count("C+m") + h[1].get("mm", "").count("C-m") > 1)
    assert n_multi == 4 and c["multi_cm"] >= n_multi
    db.free()


def test_multi_entry_records_at_scale(oracle_lib, gpu_ctx):
    """Every record of a synthetic batch re-tagged with a second C m entry
    (a C-m copy of half its calls with other ML values, placed before or after
    the C+m entry): K0 hands them to pf_k0_multi, which merges the entries'
    calls; the calls equal the oracle's (htslib semantics, parity unpinned:
    no reference fixture holds such a tag)."""
    from pomfret_amd import Config
    from tests._aln_cases import synth_aln
    aln = synth_aln(3, 30, 91)
    rng = np.random.default_rng(5)
    mm_new, ml_new = [], []
    for r in range(aln.n_recs):
        mm = bytes(aln.mm[aln.mm_off[r]:aln.mm_off[r + 1]]).decode()
        ml = aln.ml[aln.ml_off[r]:aln.ml_off[r + 1]].tolist()
        ents = [e for e in mm.split(";") if e]
        # the entry holding 5mC and its ML slice
        pos, o = None, 0
        for e in ents:
            hdr, *sk = e.split(",")
            nc = len(hdr.rstrip("?.")) - 2
            if hdr.startswith("C+") and "m" in hdr[2:]:
                pos = (e, o, nc, sk)
            o += len(sk) * nc
        if pos is None or len(pos[3]) < 2:
            mm_new.append(mm); ml_new.append(ml)
            continue
        e, o, nc, sk = pos
        # the C-m copy: every other call of the C+m entry (re-based skip counts)
        ranks = np.cumsum(np.array(sk, np.int64) + 1) - 1
        sub = ranks[::2]
        skips = np.diff(np.concatenate([[-1], sub])) - 1
        extra = "C-m?," + ",".join(str(x) for x in skips.tolist()) + ";"
        qx = rng.integers(0, 256, len(sub)).tolist()
        if r % 2:
            mm_new.append(mm + extra); ml_new.append(ml + qx)
        else:
            mm_new.append(extra + mm); ml_new.append(qx + ml)
    enc = [np.frombuffer(m.encode(), np.uint8) for m in mm_new]
    aln.mm = np.concatenate(enc)
    aln.mm_off = np.concatenate([[0], np.cumsum([len(x) for x in enc])]).astype(np.uint64)
    aln.ml = np.concatenate([np.asarray(x, np.uint8) for x in ml_new])
    aln.ml_off = np.concatenate([[0], np.cumsum([len(x) for x in ml_new])]).astype(np.uint64)
    db, _ = _check_calls(oracle_lib, gpu_ctx, Config(), LoadConfig(), aln, "multi-entry")
    assert db.load_counters()["multi_cm"] >= aln.n_recs // 2
    db.free()


def test_handmade_sequential_path(oracle_lib, gpu_ctx, monkeypatch):
    """PF_K0_PATH=seq walks every record with the literal lane-0 loop."""
    from pomfret_amd import Config
    monkeypatch.setenv("PF_K0_PATH", "seq")
    db, _ = _check_calls(oracle_lib, gpu_ctx, Config(), LOAD_CFG_SMALL, handmade_batch(), "handmade-seq")
    db.free()


def test_fatal_cigar_is_an_error(gpu_ctx):
    from pomfret_amd import Config, PomfretError
    # a CIGAR whose query length differs from SEQ is refused at upload (htslib's bam_read1 check)
    aln = records_batch([(0, 10, [dict(seq="ACGTTCGA", cigar="6M2H", mm="C+m?,0,0;", ml=[200, 10], pos=100)])])
    with pytest.raises(PomfretError):
        gpu_ctx.upload_aln(Config(), aln, LOAD_CFG_SMALL)
    # an X op the walk reaches is the reference's exit(1) (776-779): an error of the run
    aln = records_batch([(0, 10, [dict(seq="ACGTTCGA", cigar="6M2X", mm="C+m?,0,0;", ml=[200, 10], pos=100)])])
    db = gpu_ctx.upload_aln(Config(), aln, LOAD_CFG_SMALL)   # the loader runs in every run, not at upload
    with pytest.raises(PomfretError):
        db.run()
    with pytest.raises(PomfretError):
        db.debug_calls()
    db.free()


def test_arrays_grow_and_rerun(oracle_lib, gpu_ctx, monkeypatch):
    """Staging arena, call arrays and site slots sized too small at upload
    (PF_TEST_TIGHT) overflow, grow and re-run with identical results."""
    from pomfret_amd import Config, LoadConfig
    name, aln = CASES[0]
    cfg, lcfg = Config.from_coverage(30, given=False), LoadConfig()
    ref = gpu_ctx.upload_aln(cfg, aln, lcfg)
    out_ref = ref.run()
    ref.free()
    monkeypatch.setenv("PF_TEST_TIGHT", "1")
    db = gpu_ctx.upload_aln(cfg, aln, lcfg)
    out = db.run()
    for f in ("decision", "dir_table", "win_n_sites", "win_n_reads", "read_hp"):
        assert np.array_equal(getattr(out_ref, f), getattr(out, f)), f
    db.free()


@pytest.mark.parametrize("name,aln", CASES, ids=[c[0] for c in CASES])
def test_record_level_parity(oracle_lib, gpu_ctx, name, aln):
    """K0 calls, then the whole methphase result of the record-level batch."""
    from pomfret_amd import Config, LoadConfig
    cfg = Config.from_coverage(30, given=False)
    lcfg = LoadConfig()
    db, b = _check_calls(oracle_lib, gpu_ctx, cfg, lcfg, aln, name)
    ref = oracle_lib.methphase(cfg, b, n_threads=8)
    out = db.run()
    for f in ("decision", "dir_table", "dir_join", "dir_which_way", "win_n_sites", "win_n_reads", "read_hp"):
        assert np.array_equal(getattr(ref, f), getattr(out, f)), f"{name}: {f}"
    np.testing.assert_allclose(out.dir_fisher_p, ref.dir_fisher_p, rtol=1e-6, atol=0)
    out2 = db.run()                                  # K0 re-runs every launch: same result
    assert np.array_equal(out2.read_hp, out.read_hp) and np.array_equal(out2.decision, out.decision)
    db.free()


def test_scratch_trigger_lists(oracle_lib, gpu_ctx):
    """Reads with more 5mC calls than the per-wave LDS list (2048) use HBM
    scratch; aln_dense_cpg has such reads."""
    from pomfret_amd import Config, LoadConfig
    aln = dict(CASES)["aln_dense_cpg"]
    big = np.diff(aln.ml_off.astype(np.int64)) > 2048
    assert big.any()
    db, _ = _check_calls(oracle_lib, gpu_ctx, Config.from_coverage(30, given=False), LoadConfig(), aln, "dense")
    db.free()


@pytest.mark.parametrize("pad", [0x2, 0x4, 0xF])
def test_odd_length_pad_nibble(oracle_lib, gpu_ctx, pad):
    """SEQ of an odd-length record ends in a pad nibble the SAM spec leaves
    unspecified; htslib's loops (and the oracle's) stop at l_qseq, so the pad
    is never a base.  Pads set to C (2), G (4) and N (15) - the bases K0's
    count and placement look for - leave the calls unchanged."""
    from pomfret_amd import Config, LoadConfig
    from tests._aln_cases import synth_aln
    aln = synth_aln(3, 30, 23)
    lq = np.asarray(aln.l_qseq, np.int64)
    odd = np.flatnonzero(lq & 1)
    assert odd.size > 10
    seq = aln.seq.copy()
    last = aln.seq_off[odd].astype(np.int64) + (lq[odd] >> 1)
    seq[last] = (seq[last] & 0xF0) | pad
    aln.seq = seq
    db, _ = _check_calls(oracle_lib, gpu_ctx, Config(), LoadConfig(), aln, f"pad{pad}")
    db.free()


@pytest.mark.parametrize("seed", [17, 18, 19])
def test_mm_parser_fuzz(oracle_lib, gpu_ctx, seed):
    """MM/ML texts of 1-6 KB with every layout and malformation of
    mm_fuzz_batch: K0's calls equal the oracle's record for record (kept or
    dropped, positions, categories)."""
    from pomfret_amd import Config
    aln = mm_fuzz_batch(seed)
    db, b = _check_calls(oracle_lib, gpu_ctx, Config(), LOAD_CFG_SMALL, aln, f"mm-fuzz{seed}")
    assert 0 < db.n_reads < aln.n_recs
    db.free()


def test_two_contexts_launched_together(oracle_lib, gpu_ctx):
    """The bench's (and the driver's) two contexts per GPU: a record-level
    batch's windows as two batches on two contexts of device 0, launched
    together and pipelined two deep (pf_methphase_launch / _finish, as in
    bench.py), give every window the one-context run's decision, join and
    2x2 tables, and every read its tag."""
    from pomfret_amd import Config, Context, LoadConfig
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    cfg = Config.from_coverage(60, given=False)
    lcfg = LoadConfig()
    aln = make_aln_batch(AlnSpec(n_windows=12, coverage=60, gap=50_000, seed=7, gap_mix=True,
                                 skip_frac=0.1, nosite_frac=0.1))
    ref = gpu_ctx.upload_aln(cfg, aln, lcfg).run()
    nrec = np.diff(aln.win_rec_off.astype(np.int64))
    order = np.argsort(-nrec, kind="stable")
    parts = [np.sort(order[s::2]) for s in range(2)]
    ctx2 = Context(0)
    try:
        dbs = [c.upload_aln(cfg, aln.select(p.tolist()), lcfg) for c, p in zip((gpu_ctx, ctx2), parts)]
        outs = [[d.run(), d.run()] for d in dbs]
        steps = 5
        for d in dbs:
            d.launch()
        for k in range(steps):
            if k + 1 < steps:
                for d in dbs:
                    d.launch()
            for d, o in zip(dbs, outs):
                d.finish(o[k % 2])
        for p, o in zip(parts, outs):
            got = o[(steps - 1) % 2]
            assert np.array_equal(got.decision, ref.decision[p])
            assert np.array_equal(got.dir_join, ref.dir_join[p])
            assert np.array_equal(got.dir_table, ref.dir_table[p])
            assert np.array_equal(got.win_n_reads, ref.win_n_reads[p])
            ro = np.concatenate([[0], np.cumsum(ref.win_n_reads.astype(np.int64))])
            want = np.concatenate([ref.read_hp[ro[w]:ro[w + 1]] for w in p])
            assert np.array_equal(got.read_hp, want)
        for d in dbs:
            d.free()
    finally:
        ctx2.close()
