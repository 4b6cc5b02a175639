"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Integer/byte/index outputs must be bit-identical: per-window decisions, 2x2
tables, join/which_way, site counts, per-read tags, every intermediate site
array and every read's methmer list.  The floating-point internals the north
star names -- the two-sided Fisher p of each direction (FP64, blockjoin.c:3926)
and the evaluate_separation1 score (FP32) -- must agree within 1e-6 relative;
with the same host epilogue code they are in fact identical.
"""
import numpy as np
import pytest

from tests._cases import cases, synth

pytestmark = pytest.mark.gpu

CASES = cases()


def _compare(ref, out, tag):
    for name in ("decision", "dir_table", "dir_join", "dir_which_way", "win_n_sites",
                 "win_n_reads", "read_hp"):
        a, g = getattr(ref, name), getattr(out, name)
        assert np.array_equal(a, g), f"{tag}: {name} differs at {np.argwhere(a != g)[:5].tolist()}"
    np.testing.assert_allclose(out.dir_fisher_p, ref.dir_fisher_p, rtol=1e-6, atol=0, err_msg=tag)
    np.testing.assert_allclose(out.dir_score, ref.dir_score, rtol=1e-6, atol=0, err_msg=tag)


def test_division_selftest(gpu_ctx):
    """The greedy kernel divides 16-bit counts with one Newton step on the
    hardware reciprocal; it must equal correctly rounded fp32 division (the
    reference's `(float)cnt/sum` of query_counts_of_mmrs, blockjoin.c:3508-3509) for every pair.
    The DPP/permlane wave scans and group sums are checked in the same call."""
    assert gpu_ctx.selftest() == 0


@pytest.mark.parametrize("name,cfg,batch", CASES, ids=[c[0] for c in CASES])
def test_windows_parity(oracle_lib, gpu_ctx, name, cfg, batch):
    ref = oracle_lib.methphase(cfg, batch, n_threads=8)
    db = gpu_ctx.upload(cfg, batch)
    out = db.run()
    _compare(ref, out, name)
    db.free()


@pytest.mark.parametrize("name,cfg,batch", CASES, ids=[c[0] for c in CASES])
def test_sites_and_methmers_parity(oracle_lib, gpu_ctx, name, cfg, batch):
    """Intermediates: get_methmer_sites_and_ranges (both directions) and every
    read's get_mmr_of_read output (mmr_n, mmr_start_i, keys)."""
    db = gpu_ctx.upload(cfg, batch)
    ro = batch.win_read_off
    for d in (0, 1):
        n, st, keys = db.debug_methmers(d)
        k0 = 0
        for w in range(batch.n_windows):
            real, starts, lens = oracle_lib.window_sites(cfg, batch, w, d)
            g_real, g_starts, g_lens = db.debug_sites(w, d)
            assert np.array_equal(real, g_real), f"{name} w{w} d{d} sites"
            assert np.array_equal(starts, g_starts), f"{name} w{w} d{d} starts"
            assert np.array_equal(lens, g_lens), f"{name} w{w} d{d} lens"
            on, ost, okeys = oracle_lib.window_methmers(cfg, batch, w, d)
            gn = n[ro[w]:ro[w + 1]]
            assert np.array_equal(on, gn), f"{name} w{w} d{d} mmr_n {np.argwhere(on != gn)[:3]}"
            assert np.array_equal(ost, st[ro[w]:ro[w + 1]]), f"{name} w{w} d{d} mmr_start"
            assert np.array_equal(okeys, keys[k0:k0 + len(okeys)]), f"{name} w{w} d{d} keys"
            k0 += len(okeys)
        assert k0 == len(keys)
    db.free()


def test_full_size_workload(oracle_lib, gpu_ctx):
    """The bench workload (256 chr20-like windows at 30x): bit-exact against the
    oracle on every window, deterministic across runs."""
    from pomfret_amd import Config
    cfg = Config.from_coverage(30, given=False)
    b = synth(256, 30, 1000)
    ref = oracle_lib.methphase(cfg, b, n_threads=16)
    db = gpu_ctx.upload(cfg, b)
    out1 = db.run()
    out2 = db.run()
    _compare(ref, out1, "full")
    _compare(out1, out2, "rerun")
    db.free()


def test_sharding_invariance(gpu_ctx):
    """Windows are independent: any sub-batch (a GPU shard) reproduces the
    full batch's per-window results, in any window order."""
    from pomfret_amd import Config
    from pomfret_amd.shard import lpt_partition, window_costs
    cfg = Config.from_coverage(30, given=False)
    b = synth(24, 30, 77, gap_mix=True)
    full = gpu_ctx.upload(cfg, b).run()
    parts = lpt_partition(window_costs(b), 3)
    for idx in parts:
        idx = idx[::-1]
        sub = b.select(idx)
        res = gpu_ctx.upload(cfg, sub).run()
        assert np.array_equal(res.decision, full.decision[idx])
        assert np.array_equal(res.dir_table, full.dir_table[idx])
        ro = b.win_read_off
        hp = np.concatenate([full.read_hp[ro[w]:ro[w + 1]] for w in idx])
        assert np.array_equal(res.read_hp, hp)


def test_one_shot_api(oracle_lib):
    """pf_methphase_windows (upload + run + free in one call)."""
    from pomfret_amd import Config, methphase_windows
    cfg = Config.from_coverage(30, given=False)
    b = synth(4, 30, 99)
    out = methphase_windows(cfg, b, device=0)
    ref = oracle_lib.methphase(cfg, b)
    _compare(ref, out, "oneshot")


@pytest.mark.parametrize("lds", ["0", "20000"])
def test_lds_budget_variants(oracle_lib, gpu_ctx, monkeypatch, lds):
    """The greedy kernel's memory variants (tables and slot lists in LDS, tables
    in LDS with slot lists in HBM, everything in the HBM scratch arena) give
    the same bits; PF_K3_LDS caps the dynamic LDS a workgroup may take."""
    from pomfret_amd import Config
    monkeypatch.setenv("PF_K3_LDS", lds)
    cfg = Config.from_coverage(30, given=False)
    b = synth(8, 30, 41, gap_mix=True)
    ref = oracle_lib.methphase(cfg, b, n_threads=8)
    db = gpu_ctx.upload(cfg, b)
    out = db.run()
    _compare(ref, out, f"lds{lds}")
    db.free()


@pytest.mark.parametrize("env", [{"PF_K3_CACHE": "force"}, {"PF_K3_CACHE": "hbm"}, {"PF_K3_PERSIST": "1"},
                                 {"PF_K3_PERSIST": "7", "PF_K3_CACHE": "force"},
                                 {"PF_K3_CACHE": "force", "PF_K3_GCNT": "force"},
                                 {"PF_K3_LDS": "24576", "PF_K3_LDS_FB": "73728"},
                                 {"PF_K3_KDICT": "1", "PF_K3_PERSIST": "7"}],
                         ids=["cache", "hbm_lists", "one_workgroup", "seven_workgroups_cache", "cache_counts_hbm",
                              "budget_24k", "hash_dictionary"])
def test_slot_list_sources(oracle_lib, gpu_ctx, monkeypatch, env):
    """The greedy loop's slot-list sources give the same bits on every case:
    the candidate slot-list cache (round 4: the candidates' lists in LDS, the
    appended read's list loaded an iteration ahead) forced for every problem,
    the slot lists read from HBM, and the persistent main kernel with one
    and with seven workgroups walking all the problems in turn (per-problem
    state reset between problems).  Round 5: the candidate cache with the
    count table in HBM (path 6) forced for every cache problem with u8 count
    pairs, and a 24 KB budget under which problems past it take path 6 by
    themselves.  Round 6: the hash-table slot dictionary of k > 5
    (pf_k3_kdict) at the cases' own k, with seven persistent workgroups
    taking problem after problem (its slot count must reach each one)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    seen = set()
    for name, cfg, batch in CASES:
        ref = oracle_lib.methphase(cfg, batch, n_threads=8)
        db = gpu_ctx.upload(cfg, batch)
        out = db.run()
        _compare(ref, out, f"{name}/{env}")
        # the variant that ran (pf_batch_k3_paths): "force" never reads the
        # slot lists from LDS, "hbm" never runs the cache
        p = db.k3_paths()[out.win_n_sites > 0].ravel().tolist()
        seen |= set(p)
        mode = env.get("PF_K3_CACHE")
        if mode == "force":
            assert set(p) <= {2, 3, 4, 6}, (name, p)
        elif mode == "hbm":
            assert set(p) <= {3, 4}, (name, p)
        db.free()
    if env.get("PF_K3_GCNT") == "force":
        assert 6 in seen, seen
    elif env.get("PF_K3_CACHE") == "force":
        assert 2 in seen
    elif env.get("PF_K3_CACHE") == "hbm":
        assert 3 in seen


@pytest.mark.parametrize("path", ["fold", "rows"])
def test_greedy_pick_paths(oracle_lib, gpu_ctx, monkeypatch, path):
    """The greedy pick's alternatives give the same bits as the exact-interval
    pick: every pick through the sequential fp32 fold over terms recomputed
    from the tables (PF_K3_PATH=fold), and every iteration through the chunked
    record-row path with the in-LDS fold (PF_K3_PATH=rows)."""
    from pomfret_amd import Config
    monkeypatch.setenv("PF_K3_PATH", path)
    for cov, seed in ((30, 47), (60, 48)):
        cfg = Config.from_coverage(cov, given=False)
        b = synth(6, cov, seed, gap_mix=True)
        ref = oracle_lib.methphase(cfg, b, n_threads=8)
        db = gpu_ctx.upload(cfg, b)
        out = db.run()
        _compare(ref, out, f"{path}{cov}")
        db.free()


@pytest.mark.parametrize("name,cfg,batch", CASES, ids=[c[0] for c in CASES])
def test_dense_site_path(oracle_lib, gpu_ctx, monkeypatch, name, cfg, batch):
    """K12's dense site path (HBM counters over the window's position range,
    taken by windows whose range exceeds the LDS bitmaps or whose repeated
    positions overflow the LDS hash: the big windows of a gap mix), forced on
    every window of every case: identical results."""
    monkeypatch.setenv("PF_K12_DENSE", "1")
    ref = oracle_lib.methphase(cfg, batch, n_threads=8)
    db = gpu_ctx.upload(cfg, batch)
    out = db.run()
    _compare(ref, out, name + "/dense")
    # every window with a sites pass took the dense path (pf_batch_k12_paths)
    k12 = db.k12_paths()
    assert set(k12[k12 > 0].tolist()) <= {3} and (k12 == 3).sum() >= (out.win_n_sites > 0).sum()
    db.free()


@pytest.mark.parametrize("name,cfg,batch", CASES, ids=[c[0] for c in CASES])
def test_heavy_problem_split(oracle_lib, gpu_ctx, monkeypatch, name, cfg, batch):
    """The heaviest greedy problems in pf_k3_heavy on the context's second
    stream, beside the main kernel (PF_K3_HEAVY forces the 3 heaviest): the
    same results, and the heavy kernel reports its time."""
    monkeypatch.setenv("PF_K3_HEAVY", "3")
    ref = oracle_lib.methphase(cfg, batch, n_threads=8)
    db = gpu_ctx.upload(cfg, batch)
    out = db.run()
    _compare(ref, out, name + "/heavy")
    assert "pf_k3_heavy" in gpu_ctx.kernel_times()
    out2 = db.run()                                  # pipelined slots reuse the events
    _compare(ref, out2, name + "/heavy-rerun")
    db.free()


def test_wide_windows_parity(oracle_lib, gpu_ctx):
    """Windows whose call positions span more than 2^19 (the LDS bitmap
    range): 400-500 kb gaps at 20x take the dense path without any override."""
    from pomfret_amd import Config
    from pomfret_amd.synth import SynthSpec, make_batch
    cfg = Config.from_coverage(20, given=False)
    b = make_batch(SynthSpec(n_windows=3, coverage=20, seed=41, gap=450_000))
    span = [int(b.call_pos[b.read_call_off[b.win_read_off[w]]:b.read_call_off[b.win_read_off[w + 1]]].max()
                - b.call_pos[b.read_call_off[b.win_read_off[w]]:b.read_call_off[b.win_read_off[w + 1]]].min())
            for w in range(b.n_windows)]
    assert min(span) >= 1 << 19, span
    ref = oracle_lib.methphase(cfg, b, n_threads=8)
    db = gpu_ctx.upload(cfg, b)
    out = db.run()
    _compare(ref, out, "wide")
    assert (out.win_n_sites > 0).all()
    db.free()


@pytest.mark.parametrize("env", [{"PF_K12_CAP": "0"}, {"PF_K12_SMAX": "0"},
                                 {"PF_K12_CAP": "0", "PF_K2_ENTCAP": "0"}, {"PF_K12_CAP": "40"},
                                 {"PF_K12C_MINR": "1"}, {"PF_K12C_MINR": "1", "PF_K12_CAP": "40"},
                                 {"PF_K12C_MINR": "0"}],
                         ids=["all_reads_fallback", "no_lds_sites", "fallback_hbm_scratch", "mixed",
                              "all_windows_chunked", "chunked_and_fallback", "no_chunks"])
def test_methmer_fallback_paths(oracle_lib, gpu_ctx, monkeypatch, env):
    """Reads the fused sites+methmers kernel hands to the K2 fallback kernel
    (site-entry bound above its wave buffer, windows whose sites do not fit
    LDS, HBM scratch for very large reads), and windows it hands to
    pf_k12_chunks (round 5: the heavy windows' methmer phase in 64-read
    chunks over the device; PF_K12C_MINR=1 sends every window) give the same
    bits, including every read's methmer list."""
    from pomfret_amd import Config
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = Config.from_coverage(30, given=False)
    b = synth(6, 30, 43, gap_mix=True)
    ref = oracle_lib.methphase(cfg, b, n_threads=8)
    db = gpu_ctx.upload(cfg, b)
    out = db.run()
    _compare(ref, out, str(env))
    ro = b.win_read_off
    for d in (0, 1):
        n, st, keys = db.debug_methmers(d)
        k0 = 0
        for w in range(b.n_windows):
            on, ost, okeys = oracle_lib.window_methmers(cfg, b, w, d)
            assert np.array_equal(on, n[ro[w]:ro[w + 1]])
            assert np.array_equal(ost, st[ro[w]:ro[w + 1]])
            assert np.array_equal(okeys, keys[k0:k0 + len(okeys)])
            k0 += len(okeys)
    db.free()


def test_pipelined_launch_finish(oracle_lib, gpu_ctx):
    """Two runs in flight (pf_methphase_launch x2, then finish x2) give the
    same bits as pf_methphase_run; a third launch or a finish with nothing in
    flight is an argument error."""
    from pomfret_amd import Config, PomfretError
    cfg = Config.from_coverage(30, given=False)
    b = synth(6, 30, 51, gap_mix=True)
    ref = oracle_lib.methphase(cfg, b, n_threads=8)
    db = gpu_ctx.upload(cfg, b)
    db.launch()
    db.launch()
    with pytest.raises(PomfretError):
        db.launch()
    o1 = db.finish()
    o2 = db.finish()
    with pytest.raises(PomfretError):
        db.finish()
    _compare(ref, o1, "pipelined-1")
    _compare(ref, o2, "pipelined-2")
    _compare(ref, db.run(), "after")
    db.free()


@pytest.mark.parametrize("env", [{"PF_K3_IMPL": "wave"}, {"PF_K3_IMPL": "wave", "PF_K3W_LDS": "6000"},
                                 {"PF_K3_IMPL": "wave", "PF_K3W_LDS": "16384"}],
                         ids=["wave_kernel", "wave_defers_most", "wave_small_lds"])
def test_greedy_kernel_variants(oracle_lib, gpu_ctx, monkeypatch, env):
    """The main greedy kernel is the 256-thread build; PF_K3_IMPL=wave runs
    the one-wavefront build instead (fp32 lane partials, candidate slot-list
    cache, u8 count pairs), and a small PF_K3W_LDS defers its problems to the
    fallback kernel.  Every variant gives the oracle's bits."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for name, cfg, batch in [c for c in CASES if c[0] in ("synth30", "synth60", "gapmix", "oddtags", "report200")]:
        ref = oracle_lib.methphase(cfg, batch, n_threads=8)
        db = gpu_ctx.upload(cfg, batch)
        _compare(ref, db.run(), f"{name}/{env}")
        db.free()
