#!/usr/bin/env python3
"""Benchmark of the MI355X methphase hot path (BASELINE.json metric).

One "step" = one pass of the hot path over one batch of windows whose BAM
records (decoded on the host: flag, MAPQ, pos, CIGAR, 4-bit SEQ, MM/ML, de, HP)
are already resident in HBM:
  K0 loader (read filters + 5mC extraction of every record, blockjoin.c:
  1043-1173 / 794-908 / 605-792) -> K12 sites + methmers (+ K2 fallback) ->
  K3 greedy + 2x2 tables (+ K3 fallback) -> D2H -> host Fisher test, join
  decisions and read tags (pf_methphase_launch + pf_methphase_finish, two
  steps in flight).
The job: BASELINE.json's target is quoted on HG002 60x (a whole genome) at
1 GPU, so the job is WGS-sized: --tiles (8) contigs, each carrying the same
--windows (1024) distinct gap windows at 60x with SURVEY 8d's log-uniform
5-500 kb gap mix (HG002-like, synthesised -- HG002 is not available offline),
8192 windows in all; parameters as `pomfret methphase` derives them without
-c (cov_for_selection 7, cov_for_runtime 14, n_cand 16; blockjoin.c:
4373-4375), loader defaults -q 10 -L 15000, ML bands 100/156 (cli.c:52-63).
A GPU's share of the job is a list of record-level batches (<= 1024 windows
each, and at least --min-batches (2)) dealt over --split (4) contexts of the
GPU -- what the driver does with its PF_DEV_CONTEXTS contexts per GPU -- and
every step launches all of them.
The first batch alone gives the per-kernel figures and the roofline.
`--calls-level` times the previous boundary instead (reads and 5mC calls
resident, no K0).  --coverage 30 --windows 256 is configs[1]'s shape.

Multi-GPU (torchrun, one process per GPU): strong scaling by default -- the
job's windows are dealt over the ranks by the product's LPT
(pomfret_amd.shard.lpt_partition on the windows' SEQ + MM bytes), so the N=1
line is the same job as the N=8 line; no collective in the data path; after
each step the int8 decisions are all-gathered over RCCL (the drop-in's only
exchange: the host that writes VCF/GTF needs all decisions).  --weak gives
every rank a whole job of its own.  At N=1 the `strong_projection` leg times
rank 0's share of the same job at N=2/4/8 on this GPU, and `critical_window`
the heaviest window alone (the floor of any GPU's step).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_HBM_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# N=1 headline: BASELINE.json's target is quoted on HG002 60x at 1 GPU.  Gap
# lengths log-uniform 5-500 kb (SURVEY.md 8d's mix); as in real runs some
# windows are skipped (left-block reads mostly untagged: 1161-1163) or have
# no qualifying site (4266).  --workload fixed50: round 2's 50 kb windows.
WORKLOADS = {
    "mix": dict(n_windows=1024, coverage=60, gap=50_000, gap_mix=True, skip_frac=0.10, nosite_frac=0.05),
    "fixed50": dict(n_windows=1024, coverage=60, gap=50_000, gap_mix=False, skip_frac=0.0, nosite_frac=0.0),
}
WORKLOAD = WORKLOADS["mix"]
CPU_SHARE = 16           # host cores per GPU on the MI355X boxes (OMP_NUM_THREADS there)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algo_bytes(batch, stats, n_sites, heavy=()):
    """Algorithmic bytes per launch of each kernel.

    K12 sites + methmers (fused; the K2 kernel only takes fallback reads,
                 usually none, and is credited 0 B):
                 5 B per call read (u32 pos + u8 cat) + 9 B per site written,
                 and per (read, dir) 5 B per call read, 4 B per site entry
                 read (~ one per methmer) and 4 B per methmer key written
    K3 greedy  : 12 B per methmer lookup (4 B key + 2x(2 B cnt + 2 B sum)),
                 8 B per methmer inserted, 1 B per read visited by the scan,
                 2 B per strict reference read in the 2x2 table
    """
    N = batch.n_calls
    S = int(n_sites.sum())
    lookups = int(stats[:, :, 0].sum())
    inserts = int(stats[:, :, 1].sum())
    scanned = int(stats[:, :, 3].sum())
    mmr = int(stats[:, :, 4].sum())
    strict = int(stats[:, :, 5].sum())
    k1 = 5 * N + 9 * S
    k2 = 2 * 5 * N + 8 * mmr          # calls read per direction + sites read / methmers written
    k3 = 12 * lookups + 8 * inserts + scanned + 2 * strict
    # the problems pf_k3_heavy runs (pf_batch_heavy) are credited to it
    hv = np.zeros(stats.shape[:2], bool)
    for p in heavy:
        hv[int(p) >> 1, int(p) & 1] = True
    st_h = stats[hv]
    k3h = int(12 * st_h[:, 0].sum() + 8 * st_h[:, 1].sum() + st_h[:, 3].sum() + 2 * st_h[:, 5].sum()) if len(st_h) else 0
    # fallback kernels (pf_k2_methmers, pf_k3_fallback) take the rare oversize reads
    # and problems, none on this workload: credited 0 B
    return {"pf_k12_sites_methmers": k1 + k2, "pf_k2_methmers": 0, "pf_k3_greedy": k3 - k3h, "pf_k3_heavy": k3h,
            "pf_k3_fallback": 0}


def k0_bytes(aln, read_recs, n_calls):
    """Algorithmic bytes per launch of K0: per record 15 B of
    filter fields (wave-slot index, flag, MAPQ, l_qseq, de) read and 4 B
    (rec_n) written; per kept record 55 B of fixed fields (pos, the record's
    offsets), its CIGAR (4 B/op), 4-bit SEQ (l_qseq/2 B) and MM text read and
    24 B written (start, end, first, last, staging offset); per call 1 B of ML
    read and 5 B (u32 pos + u8 cat) written to its staging slice."""
    kept = np.asarray(read_recs, np.int64)
    cig = np.diff(aln.cigar_off.astype(np.int64))[kept]
    mm = np.diff(aln.mm_off.astype(np.int64))[kept]
    seq = (aln.l_qseq.astype(np.int64)[kept] + 1) // 2
    R = kept.shape[0]
    return int(19 * aln.n_recs + 79 * R + 4 * cig.sum() + seq.sum() + mm.sum() + 6 * n_calls)


def pack_bytes(n_recs, R, n_calls):
    """scan + pack: 4 B (rec_n) per record; per kept read 25 B read (record
    fields, staging offset, HP) and 34 B written (read fields, record index,
    two tag copies, call offset); per call 5 B read + 5 B written."""
    return int(4 * n_recs + 59 * R + 10 * n_calls)


def pmc_traffic(kernel: str, wl: dict, boundary: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py) when it was
    collected on this run's workload `wl` and boundary, or None."""
    p = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") != dict(wl, boundary=boundary):
            return None
        return d["kernels"].get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def record_spans(aln, recs):
    """(pos, bam_endpos) of the records `recs`: pos + the reference-consuming
    CIGAR lengths (M, D, N, =, X)."""
    cig = np.asarray(aln.cigar, np.uint32)
    ref = np.where(np.isin(cig & 15, (0, 2, 3, 7, 8)), cig >> 4, 0).astype(np.uint64)
    cs = np.concatenate([[0], np.cumsum(ref)])
    off = np.asarray(aln.cigar_off, np.int64)
    recs = np.asarray(recs, np.int64)
    start = np.asarray(aln.pos, np.uint32)[recs]
    rlen = cs[off[recs + 1]] - cs[off[recs]]
    return start, (start + rlen).astype(np.uint32)


def cpu_baseline(cfg, batch, threads: int, min_cpu_s: float = 20.0, max_reps: int = 200):
    """The CPU oracle (plain-C restatement of the reference, oracle/) timed on
    this host with `threads` pthreads over windows (kt_for analogue): whole
    passes over the same batch until about `min_cpu_s` seconds of CPU work
    (wall x threads) are done -- a bounded sample, reported as reads/s."""
    import oracle
    oracle.methphase(cfg, batch.select(range(min(8, batch.n_windows))), n_threads=threads)
    t0 = time.perf_counter()
    reps = 0
    while reps < max_reps:
        oracle.methphase(cfg, batch, n_threads=threads)
        reps += 1
        if (time.perf_counter() - t0) * threads >= min_cpu_s and reps >= 3:
            break
    dt = time.perf_counter() - t0
    return batch.n_reads * reps / dt, dt, reps


def effective_cores():
    """(cores this process may run on, how that was found): the smaller of the
    CPU affinity set and the cgroup CPU quota (cpu.max, v2; cfs_quota_us /
    cfs_period_us, v1) -- `nproc` on the GPU box shows the whole machine."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    eff = aff if quota is None else max(1, min(aff, int(quota)))
    return eff, {"affinity": aff, "cgroup_quota_cores": round(quota, 2) if quota is not None else None}


def cpu_baseline_aln(cfg, lcfg, aln, n_reads, threads: int, min_cpu_s: float = 20.0, max_reps: int = 200,
                     min_reps: int = 2):
    """Record-level CPU path of the oracle (per window: loader + worker, the
    reference's structure), `threads` pthreads over windows, bounded sample."""
    import oracle
    t0 = time.perf_counter()
    reps = 0
    ref = None
    while reps < max_reps:
        ref = oracle.methphase_aln(cfg, lcfg, aln, n_threads=threads)
        reps += 1
        if (time.perf_counter() - t0) * threads >= min_cpu_s and reps >= min_reps:
            break
    dt = time.perf_counter() - t0
    return n_reads * reps / dt, dt, reps, ref


def e2e_leg(ctx, cfg, lcfg, wl, n_windows: int, threads: int, workdir: str, cpu: bool = True, cpu_threads: int = 0):
    """End to end from files (never `value`): the first n_windows windows of
    the workload written as a BAM + BAI (QUAL strings included, zlib level 6,
    tests/_bamio.py's writer), then per path the wall time from the BAM file to
    decisions on the host:
      device_fetch: BAI plan + compressed blocks read on the host, inflate /
                    record chain / window fetch / gather / K0..K3 on the GPU
                    (pf_batch_upload_bam + pf_methphase_run);
      host_fetch:   the host reader inflates and decodes (pf_bam_fetch_windows,
                    `threads` threads), upload_aln, K0..K3;
      cpu_port:     the host reader + the oracle's record-level path on
                    `cpu_threads` threads (the reference's structure: htslib
                    decode + the kt_for worker)."""
    cpu_threads = cpu_threads or threads
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import _bamio
    from pomfret_amd.bam import BamFile
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    t = time.perf_counter()
    aln = make_aln_batch(AlnSpec(n_windows=n_windows, coverage=wl["coverage"], gap=wl["gap"], seed=1000,
                                 gap_mix=wl["gap_mix"], skip_frac=wl["skip_frac"], nosite_frac=wl["nosite_frac"]),
                         workers=threads)
    recs = _bamio.records_from_aln(aln, qual=True)
    path = os.path.join(workdir, f"pf_e2e_{os.getpid()}.bam")
    _bamio.write_bam(path, [("chrS", 2_000_000_000)], recs, workers=threads, level=6)
    del recs
    gen_s = time.perf_counter() - t
    ws, we = aln.win_start, aln.win_end
    res = {"windows": n_windows, "records": int(aln.n_recs), "bam_bytes": os.path.getsize(path),
           "threads": threads, "gen_s": round(gen_s, 1)}
    try:
        with BamFile(path) as b:
            dev = None
            for rep in range(2):                        # the second (warm) pass is reported
                t0 = time.perf_counter()
                db, qn, info = b.fetch_windows_device(ctx, cfg, "chrS", ws, we, lcfg)
                t1 = time.perf_counter()
                out = db.run()
                t2 = time.perf_counter()
                reads = int(out.win_n_reads.sum())
                dec_dev = out.decision.copy()
                db.free()
                dev = {"reads_per_s": round(reads / (t2 - t0), 1), "ms": round((t2 - t0) * 1e3, 1),
                       "fetch_ms": round((t1 - t0) * 1e3, 1), "run_ms": round((t2 - t1) * 1e3, 1),
                       "inflate_ms": round(info["ms_inflate"], 2), "read_ms": round(info["ms_read"], 1),
                       "chain_ms": round(info["ms_chain"], 2), "decode_ms": round(info["ms_decode"], 2),
                       "select_ms": round(info["ms_select"], 2), "build_ms": round(info["ms_build"], 1),
                       "compressed_bytes": int(info["comp_bytes"]), "inflated_bytes": int(info["inflated_bytes"]),
                       "inflate_GBps": round(info["inflated_bytes"] / max(info["ms_inflate"], 1e-6) / 1e6, 2)}
            res["reads"] = reads
            res["device_fetch"] = dev
            t0 = time.perf_counter()
            got, qn_h, _ = b.fetch_windows("chrS", ws, we, threads=threads)
            t1 = time.perf_counter()
            db = ctx.upload_aln(cfg, got, lcfg)
            out = db.run()
            t2 = time.perf_counter()
            db.free()
            res["host_fetch"] = {"reads_per_s": round(reads / (t2 - t0), 1), "ms": round((t2 - t0) * 1e3, 1),
                                 "fetch_ms": round((t1 - t0) * 1e3, 1), "upload_run_ms": round((t2 - t1) * 1e3, 1)}
            res["decisions_match"] = bool(np.array_equal(out.decision, dec_dev))
            # the pass over the whole BAM that runs without -c pay first
            # (estimate_read_coverage_dirtyfast): device fetch vs the host pass
            # with cpu_threads BGZF inflate threads (the reference's -t N: bgzf_mt)
            c0 = time.perf_counter()
            cov_d = b.estimate_coverage_device(ctx)
            c1 = time.perf_counter()
            with BamFile(path, threads=cpu_threads) as bh:
                cov_h = bh.estimate_coverage()
            c2 = time.perf_counter()
            res["coverage_estimate"] = {"device_ms": round((c1 - c0) * 1e3, 1), "host_ms": round((c2 - c1) * 1e3, 1),
                                        "host_inflate_threads": cpu_threads,
                                        "match": cov_d == cov_h, "cov": int(cov_d[0])}
            # the whole driver, file to .mp.vcf/.mp.gtf (pf_methphase_main: VCF
            # gaps, plan, jobs, first-wins tables, writers), device fetch vs
            # --host-fetch, with the run's parameters given (the coverage
            # estimate a run without -c adds is timed above)
            from pomfret_amd.pipeline import methphase_files
            vcf = path[:-4] + ".vcf"
            _bamio.write_phased_vcf(vcf, "chrS", list(zip(ws.tolist(), we.tolist())), chrom_len=2_000_000_000)
            drv = {}
            for hf in (False, True):
                pre = path[:-4] + f".drv{int(hf)}"
                d0 = time.perf_counter()
                r = methphase_files(path, vcf, pre, cfg, lcfg, ctx=ctx, threads=threads, host_fetch=hf)
                d1 = time.perf_counter()
                outs = [open(pre + e, "rb").read() for e in (".mp.vcf", ".mp.gtf")]
                for e in (".mp.vcf", ".mp.gtf"):
                    os.unlink(pre + e)
                drv[hf] = (d1 - d0, r["decision"], outs)
            res["driver"] = {"device_fetch_ms": round(drv[False][0] * 1e3, 1),
                             "device_fetch_reads_per_s": round(reads / drv[False][0], 1),
                             "host_fetch_ms": round(drv[True][0] * 1e3, 1),
                             "host_fetch_reads_per_s": round(reads / drv[True][0], 1),
                             "outputs_identical": drv[False][2] == drv[True][2],
                             "decisions_match": bool(np.array_equal(drv[False][1], dec_dev)),
                             "what": "methphase_files: BAM + phased VCF -> .mp.vcf/.mp.gtf, parameters given"}
            os.unlink(vcf)
            if cpu:
                import oracle
                t5 = time.perf_counter()
                got, _, _ = b.fetch_windows("chrS", ws, we, threads=cpu_threads)
                t3 = time.perf_counter()
                ref = oracle.methphase_aln(cfg, lcfg, got, n_threads=cpu_threads)
                t4 = time.perf_counter()
                res["cpu_port"] = {"reads_per_s": round(reads / (t4 - t5), 1),
                                   "ms": round((t4 - t5) * 1e3, 1), "threads": cpu_threads,
                                   "fetch_ms": round((t3 - t5) * 1e3, 1), "worker_ms": round((t4 - t3) * 1e3, 1),
                                   "what": f"host fetch ({cpu_threads} threads) + oracle record-level worker "
                                           f"({cpu_threads} threads)"}
                res["decisions_match"] = res["decisions_match"] and bool(np.array_equal(ref.decision, dec_dev))
    finally:
        os.unlink(path)
        if os.path.exists(path + ".bai"):
            os.unlink(path + ".bai")
    return res


def k4_bytes(known, reads) -> int:
    """SURVEY.md 8d's -u bytes: per read 4 n_cigar + (l_MD + 1) + n_X +
    n_I_bases + 16 V_known_in_span + 1."""
    cig = np.asarray(reads.cigar, np.uint32)
    kp = np.asarray(known.pos, np.int64)
    v_span = int((np.searchsorted(kp, np.asarray(reads.end, np.int64))
                  - np.searchsorted(kp, np.asarray(reads.start, np.int64))).sum())
    md = np.asarray(reads.md, np.uint8)
    n_x = int(np.isin(md, np.frombuffer(b"ACGT", np.uint8)).sum())
    ins = int((cig[(cig & 15) == 1] >> 4).sum())
    return int(4 * cig.shape[0] + md.shape[0] + reads.n_reads + n_x + ins + 16 * v_span + reads.n_reads)


def e2e_u_leg(ctx, lcfg, threads: int, workdir: str, scale: float = 1.0, cpu: bool = True, cpu_threads: int = 0):
    """BASELINE configs[3]'s shape from files (never `value`): `pomfret
    methphase -u` without -c on a whole-genome-shaped 60x BAM (tests/_genome:
    4 contigs, reads uniform over each contig, ~1,000 phase-block gaps of
    5-40 kb between 50-100 kb blocks, 5 % short blocks merged away, het SNVs
    1/kb with MD:Z, no HP, QUAL strings, zlib level 6), timed file to
    .mp.vcf/.mp.gtf:
      cli:      the pomfret-amd binary as a user runs it (process start, HIP
                init, the device coverage pass, the device -u pre-pass over
                every primary read, the window jobs, the writers);
      driver:   the same driver in this process on a warm context;
      cpu_port: the product's planner / writers with the host reader (its
                coverage pass and -u contig reads with BGZF inflate threads,
                the reference's -t N bgzf_mt) and the oracle computing every
                job (tests/_oracle_pipeline.methphase_files_port,
                `cpu_threads` threads);
    outputs compared byte for byte.  Also the K4 kernel on the largest
    contig's reads (HIP events, SURVEY 8d's -u bytes)."""
    import subprocess
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import _genome
    cpu_threads = cpu_threads or threads
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from pomfret_amd.pipeline import methphase_files
    spec = _genome.GenomeSpec()
    spec.contigs = tuple((n, int(L * scale)) for n, L in spec.contigs)
    prefix = os.path.join(workdir, f"pf_e2eu_{os.getpid()}")
    t = time.perf_counter()
    g = _genome.write_genome(prefix, spec, workers=threads)
    res = {"contigs": len(spec.contigs), "genome_bp": int(sum(L for _, L in spec.contigs)),
           "coverage": spec.coverage, "records": g["n_records"],
           "bam_bytes": g["bam_bytes"], "known_snvs": g["n_snvs"], "threads": threads,
           "gen_s": round(time.perf_counter() - t, 1)}
    log(f"[bench] e2e_u: generated {res['records']} records, {res['bam_bytes'] / 1e9:.2f} GB in {res['gen_s']}s")
    outs = {}

    def take(pre):
        o = [open(pre + e, "rb").read() for e in (".mp.vcf", ".mp.gtf")]
        for e in (".mp.vcf", ".mp.gtf"):
            os.unlink(pre + e)
        return o

    try:
        cli = os.path.join(HERE, "pomfret_amd", "pomfret-amd")
        cmd = [cli, "methphase", "-u", "-t", str(threads), "-o", prefix + ".cli", "--vcf", g["vcf"], g["bam"]]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, capture_output=True, text=True)
        t1 = time.perf_counter()
        if p.returncode != 0:
            raise RuntimeError(f"pomfret-amd failed ({p.returncode}): {p.stderr[-2000:]}")
        outs["cli"] = take(prefix + ".cli")
        log(f"[bench] e2e_u: cli {t1 - t0:.2f}s")
        # what chromosome-scale contigs cost, on this genome: (a) no kept
        # arenas (a contig whose inflated BAM would break the HBM reserve:
        # its window jobs re-read and re-inflate their ranges), (b) the -u
        # pre-pass in position pieces of 256 MiB compressed (a 60x chr1 is
        # tens of GB: pieces of 4 GiB), outputs compared with the others
        variants = {}
        for key, extra in (("cli_no_kept_arenas", {"PF_FETCH_CACHE": "0"}),
                           ("cli_pieces_256MiB", {"PF_FETCH_PIECE_BYTES": str(256 << 20)})):
            tv = time.perf_counter()
            pv = subprocess.run([c if c != prefix + ".cli" else prefix + "." + key for c in cmd], capture_output=True,
                                text=True, env=dict(os.environ, **extra))
            dv = time.perf_counter() - tv
            if pv.returncode != 0:
                raise RuntimeError(f"pomfret-amd ({key}) failed ({pv.returncode}): {pv.stderr[-2000:]}")
            outs[key] = take(prefix + "." + key)
            variants[key] = {"s": round(dv, 2), "env": extra}
            log(f"[bench] e2e_u: {key} {dv:.2f}s")
        t0d = time.perf_counter()
        r = methphase_files(g["bam"], g["vcf"], prefix + ".drv", None, lcfg, ctx=ctx, untagged=True, threads=threads)
        t1d = time.perf_counter()
        outs["driver"] = take(prefix + ".drv")
        dec = r["decision"]
        res["windows"] = int(dec.shape[0])
        res["decisions"] = {"cis": int((dec == 0).sum()), "trans": int((dec == 1).sum()),
                            "none": int((dec < 0).sum())}
        res["raw_tags"] = len(r["raw_hp"])
        log(f"[bench] e2e_u: driver {t1d - t0d:.2f}s, {res['windows']} windows")
        res["cli"] = {"s": round(t1 - t0, 2), "records_per_s": round(res["records"] / (t1 - t0), 1),
                      "what": " ".join(["pomfret-amd", "methphase", "-u", "-t", str(threads), "-o", "P",
                                        "--vcf", "V", "B"])}
        res["cli_variants"] = variants
        res["driver"] = {"s": round(t1d - t0d, 2), "records_per_s": round(res["records"] / (t1d - t0d), 1),
                         "phases": r["stats"], "what": "methphase_files in this process, warm context"}
        # K4 on the largest contig (the -u pre-pass's kernel, warm)
        name = max(spec.contigs, key=lambda c: c[1])[0]
        kv = vcf_known_vars(g["vcf"], name)
        with BamFile(g["bam"]) as b:
            b.haptag_device(ctx, name, kv)
            t0k = time.perf_counter()
            hp, qn, info = b.haptag_device(ctx, name, kv)
            t1k = time.perf_counter()
            kt = ctx.kernel_times()
            kname = next((k for k in kt if k.startswith("pf_k4")), None)
            reads, _, _ = b.fetch_contig_reads(name)
        kms = kt.get(kname, float("nan"))
        ab = k4_bytes(kv, reads)
        res["k4"] = {"kernel": kname, "contig": name, "reads": int(reads.n_reads), "known": int(len(kv.pos)),
                     "ms": round(kms, 4), "reads_per_s": round(reads.n_reads / (kms * 1e-3), 1),
                     "algo_bytes": ab, "GBps": round(ab / (kms * 1e-3) / 1e9, 2),
                     "prepass_ms": round((t1k - t0k) * 1e3, 1), "inflate_ms": round(info["ms_inflate"], 2),
                     "inflated_bytes": int(info["inflated_bytes"])}
        log(f"[bench] e2e_u: k4 {json.dumps(res['k4'])}")
        if cpu:
            from _oracle_pipeline import methphase_files_port
            rp, ph = methphase_files_port(g["bam"], g["vcf"], prefix + ".port", None, lcfg, untagged=True,
                                          threads=cpu_threads)
            outs["cpu_port"] = take(prefix + ".port")
            res["cpu_port"] = {"s": round(ph["total_s"], 2), "records_per_s": round(res["records"] / ph["total_s"], 1),
                               "phases_s": {k: round(v, 2) for k, v in ph.items() if k != "total_s"},
                               "threads": cpu_threads,
                               "what": f"host reader (coverage pass and -u contig reads with BGZF inflate threads) + "
                                       f"oracle jobs, {cpu_threads} threads (-t {cpu_threads})"}
            res["vs_cpu_port"] = round(ph["total_s"] / (t1 - t0), 2)
        res["outputs_identical"] = all(o == outs["cli"] for o in outs.values())
        res["compared"] = sorted(outs)
    finally:
        for f in (g["bam"], g["bam"] + ".bai", g["vcf"]):
            if os.path.exists(f):
                os.unlink(f)
    return res


def stagger_groups(groups, gctx, split: int, base_costs):
    """The contexts out of phase: context c > 0 runs its first batch as two
    halves (dealt heaviest first, round-robin), so its later batches start
    half a batch after context 0's -- one context's K3 tail (few long greedy
    problems) then runs beside another's K0 / K12 instead of beside its
    twin's tail.  Same windows, same batches otherwise."""
    out_g, out_c, done = [], [], set()
    for g, c in zip(groups, gctx):
        if c > 0 and c not in done and g[1].shape[0] >= 2:
            done.add(c)
            order = np.argsort(-np.asarray(base_costs, np.float64)[g[1]], kind="stable")
            for h in (order[0::2], order[1::2]):
                h = np.sort(h)
                out_g.append((g[0][h], g[1][h]))
                out_c.append(c)
        else:
            out_g.append(g)
            out_c.append(c)
    return out_g, out_c


def oracle_sample(aln, gaps, n_reads_w, n: int = 64):
    """The cpu_baseline sample: the heaviest windows (most kept reads), the
    widest gaps (>= 400 kb: K12's dense site path), then the first windows,
    up to n windows in all (sorted)."""
    heavy = np.argsort(-np.asarray(n_reads_w, np.int64), kind="stable")[:8]
    wide = [int(w) for w in np.argsort(-np.asarray(gaps, np.int64), kind="stable")[:4] if gaps[w] >= 400_000]
    pick = list(dict.fromkeys([int(w) for w in heavy] + wide))
    for w in range(aln.n_windows):
        if len(pick) >= n:
            break
        if w not in pick:
            pick.append(w)
    return sorted(pick[:n])


def compare_with_oracle(out, wro, ref, sub, tags: bool = True):
    """GPU result `out` of a batch (window read offsets `wro`) against the
    oracle's result `ref` of the windows `sub`: decisions, 2x2 tables, joins,
    site and read counts and read tags bit for bit, Fisher p at rtol 1e-6."""
    wro = np.asarray(wro, np.int64)
    sub = np.asarray(sub, np.int64)
    bad = []
    for f in ("decision", "dir_table", "dir_join", "dir_which_way", "win_n_sites", "win_n_reads", "dir_score"):
        if not np.array_equal(getattr(out, f)[sub], getattr(ref, f)):
            bad.append(f)
    hp = np.concatenate([out.read_hp[wro[w]:wro[w + 1]] for w in sub]) if sub.size else np.zeros(0, np.uint8)
    if tags and not np.array_equal(hp, ref.read_hp):
        bad.append("read_hp")
    p, q = out.dir_fisher_p[sub], ref.dir_fisher_p
    if not np.all(np.abs(p - q) <= 1e-6 * np.abs(q)):
        bad.append("dir_fisher_p")
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--windows", type=int, default=WORKLOAD["n_windows"],
                    help="base windows (distinct); the job is --tiles copies of them")
    ap.add_argument("--tiles", type=int, default=8,
                    help="the job: this many copies of the base windows, each copy a contig of its own "
                         "(8 x 1024 = 8192 windows: a WGS-sized job)")
    ap.add_argument("--coverage", type=int, default=WORKLOAD["coverage"])
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="mix",
                    help="mix: log-uniform 5-500 kb gaps with skipped / site-less windows; fixed50: 50 kb gaps")
    ap.add_argument("--weak", action="store_true",
                    help="every rank runs a whole job of its own (seeds differ per rank) instead of its LPT "
                         "share of one job")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the calls-level, fixed-gap, projection, PCIe-inclusive and end-to-end legs")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--e2e-windows", type=int, default=64,
                    help="windows of the end-to-end (BAM file -> decisions) leg; 0 skips it")
    ap.add_argument("--e2e-u-scale", type=float, default=1.0,
                    help="genome scale of the configs[3]-shaped -u leg (1.0: 96 Mb, ~1,000 windows); 0 skips it")
    ap.add_argument("--split", type=int, default=4,
                    help="contexts per GPU (the driver's PF_DEV_CONTEXTS): the rank's batches are dealt over "
                         "them and launched together every step (round 6: 4, since a context's second stream "
                         "is created on first use and four contexts fit the device's four hardware queues)")
    ap.add_argument("--min-batches", type=int, default=2,
                    help="a share of fewer batches is cut into this many (a 1024-window share at N=8: two "
                         "512-window batches, not four of 256)")
    ap.add_argument("--stagger", type=int, default=0,
                    help="1: every context but the first starts with its first batch cut in two halves, so "
                         "the contexts' kernels run out of phase (round 5: 117.1 vs 114.0 ms per step, slower; off)")
    ap.add_argument("--calls-level", action="store_true",
                    help="time the calls-level boundary (reads + 5mC calls resident, no K0)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from pomfret_amd import Config, Context, LoadConfig, WindowBatch
    from pomfret_amd.shard import aln_window_costs, group_copies, lpt_bound, lpt_partition, split_groups
    from pomfret_amd.synth import SynthSpec, make_batch
    from dataclasses import replace
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch, window_cost_estimates

    wl = dict(WORKLOADS[args.workload], n_windows=args.windows, coverage=args.coverage)
    cfg = Config.from_coverage(wl["coverage"], given=False)
    lcfg = LoadConfig()
    record_level = not args.calls_level
    n_base, tiles = wl["n_windows"], max(1, args.tiles)
    n_job = n_base * tiles
    split = max(1, args.split)
    seed = 1000 + (rank if args.weak else 0)
    spec = AlnSpec(n_windows=n_base, coverage=wl["coverage"], gap=wl["gap"], seed=seed, gap_mix=wl["gap_mix"],
                   skip_frac=wl["skip_frac"], nosite_frac=wl["nosite_frac"])
    t = time.perf_counter()
    if record_level:
        # generated (in worker processes) before anything touches the GPU;
        # PF_BENCH_ALN_CACHE: a batch saved beforehand (tools/run_aln_once.py,
        # same spec), so that a traced run forks no generator workers
        cache = os.environ.get("PF_BENCH_ALN_CACHE")
        if cache and os.path.exists(cache) and not args.weak:
            from pomfret_amd.synth_aln import load_aln
            aln = load_aln(cache)
            assert aln.n_windows == n_base, "PF_BENCH_ALN_CACHE holds another batch"
        else:
            aln = make_aln_batch(spec, workers=0 if world == 1 else max(1, CPU_SHARE // 2))
        log(f"[bench] rank {rank}: generated {aln.n_windows} base windows, {aln.n_recs} BAM records "
            f"({aln.nbytes() / 1e9:.2f} GB) in {time.perf_counter() - t:.1f}s")
        base_costs = aln_window_costs(aln)
    else:
        cbatch = make_batch(SynthSpec(n_windows=n_base, coverage=wl["coverage"], gap=wl["gap"], seed=seed))
        from pomfret_amd.shard import window_costs
        base_costs = window_costs(cbatch)
    gaps = (aln.win_end.astype(np.int64) - aln.win_start.astype(np.int64)) if record_level else None

    # The job: `tiles` copies of the base windows, one contig each.  Strong
    # scaling (default): the job's windows are dealt over the ranks by the
    # product's LPT (pomfret_amd.shard, on the windows' SEQ + MM bytes); weak
    # (--weak): every rank runs a whole job of its own.
    job_costs = np.tile(base_costs, tiles)
    if args.weak:
        share = np.arange(n_job)
        loads = None
    else:
        parts = lpt_partition(job_costs, world)
        share = parts[rank]
        loads = [float(job_costs[p].sum()) for p in parts]
    min_batches = max(1, min(args.min_batches, split))
    groups = split_groups(group_copies(share, n_base), min_batches, base_costs)
    gctx = [gi % split for gi in range(len(groups))]
    if args.stagger and split > 1 and len(groups) > split:
        groups, gctx = stagger_groups(groups, gctx, split, base_costs)

    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend="nccl")
        dist = tdist
    ctxs = [Context(local_rank) for _ in range(split)]
    ctx = ctxs[0]
    ident = np.arange(n_base)

    def upload(c, basew):
        if record_level:
            if basew.shape[0] == n_base and np.array_equal(basew, ident):
                return c.upload_aln(cfg, aln, lcfg), aln
            sub = aln.select(basew)
            return c.upload_aln(cfg, sub, lcfg), sub
        return c.upload(cfg, cbatch.select(basew) if not np.array_equal(basew, ident) else cbatch), None

    t = time.perf_counter()
    dbs, subs = [], []
    for gi, (_, basew) in enumerate(groups):
        d, s = upload(ctxs[gctx[gi]], basew)
        dbs.append(d)
        subs.append(s if gi == 0 else None)          # the first batch's records feed the byte model
    log(f"[bench] rank {rank}: {len(share)} of {n_job} job windows as {len(dbs)} batches on {split} contexts "
        f"(upload: validation, SEQ repack, H2D; no device work): {time.perf_counter() - t:.1f}s")
    db = dbs[0]
    aln0 = subs[0]
    if record_level:
        off, cpos, ccat, _, _ = db.debug_calls()
        rr = db.read_recs()
        # the loaded reads as a window batch (the byte model and the calls-level
        # leg): K0's calls, and the spans of the kept records (pos, bam_endpos)
        wro = np.searchsorted(rr, aln0.win_rec_off.astype(np.int64)).astype(np.uint32)
        rs, re_ = record_spans(aln0, rr)
        batch = WindowBatch(win_start=aln0.win_start, win_end=aln0.win_end, win_read_off=wro,
                            read_start=rs, read_end=re_,
                            read_hp=aln0.hp[rr], read_call_off=off, call_pos=cpos, call_cat=ccat,
                            win_cov_sel=aln0.win_cov_sel, win_cov_rt=aln0.win_cov_rt, win_n_cand=aln0.win_n_cand)
        del off, cpos, ccat
    else:
        batch = cbatch.select(groups[0][1])

    def timed(dbs_, steps=None):
        """W warmup runs, then exactly K timed steps between barrier + sync
        pairs; returns (max-over-ranks seconds, reads over all ranks and
        steps, per-kernel ms summed over the steps, one step's results per
        batch).  dbs_: the batches, dealt over the contexts; every step
        launches all of them (a context runs its batches in order on its
        stream) and the steps are pipelined two deep."""
        steps = args.steps if steps is None else steps
        outs = [[d.run(), d.run()] for d in dbs_]
        n_reads = sum(int(o[0].win_n_reads.sum()) for o in outs)
        n_win = sum(d.n_windows for d in dbs_)
        for _ in range(args.warmup):
            for d in dbs_:
                d.launch()
            for d, o in zip(dbs_, outs):
                d.finish(o[0])
        use_dist = dist is not None and steps == args.steps
        if use_dist:
            import torch
            n_max = torch.tensor([n_win], dtype=torch.int64, device=f"cuda:{local_rank}")
            dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
            dec_t = torch.full((int(n_max.item()),), -2, dtype=torch.int8, device=f"cuda:{local_rank}")
            gathered = torch.empty(world * dec_t.numel(), dtype=torch.int8, device=f"cuda:{local_rank}")

        # Steps are pipelined two deep (pf_methphase_launch / _finish): the host
        # epilogue of step k (Fisher tests, decisions, read tags) overlaps the
        # kernels of step k+1; every step runs every kernel (K0 loader, scan +
        # pack, K12, K2, K3), the D2H copy and the epilogue inside the timed
        # region.  After each step the int8 decisions are all-gathered over
        # RCCL (the drop-in's only exchange: the writer needs every decision).
        def finish(k):
            for d, o in zip(dbs_, outs):
                d.finish(o[k % 2])
            if use_dist:
                dec = np.concatenate([o[k % 2].decision for o in outs])
                dec_t[:n_win].copy_(torch.from_numpy(dec))
                dist.all_gather_into_tensor(gathered, dec_t)

        if use_dist:
            dist.barrier()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        kern_acc = {}
        if steps:
            for d in dbs_:
                d.launch()
        for k in range(steps):
            if k + 1 < steps:
                for d in dbs_:
                    d.launch()
            finish(k)
            if len(dbs_) == 1:
                for kn, v in dbs_[0].ctx.kernel_times().items():
                    kern_acc[kn] = kern_acc.get(kn, 0.0) + v
        if use_dist:
            torch.cuda.synchronize()
            dist.barrier()
        elapsed = time.perf_counter() - t0
        total = float(n_reads) * steps
        if use_dist:
            tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
            rt = torch.tensor([n_reads], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(rt)
            total = float(rt.item()) * steps
        return elapsed, total, kern_acc, [o[(steps - 1) % 2] if steps else o[0] for o in outs]

    # 1. the first batch alone on one context: the per-kernel figures and the roofline
    el1, tot1, kern_acc, outs1 = timed([db])
    out = outs1[0]
    single = {"value": round(tot1 / el1, 1), "ms_per_step": round(el1 / args.steps * 1e3, 4),
              "windows": int(db.n_windows), "reads": int(out.win_n_reads.sum()),
              "what": "the rank's first batch alone on one context (kernels and roofline measured here)"}
    log(f"[bench] single batch: {json.dumps(single)}")
    stats = db.stats()
    kmean = {k: v / args.steps for k, v in kern_acc.items()}
    ab = algo_bytes(batch, stats, out.win_n_sites, db.heavy_problems())
    if record_level:
        ab["pf_k0_load"] = k0_bytes(aln0, rr, batch.n_calls)
        ab["pf_k0_pack"] = pack_bytes(aln0.n_recs, batch.n_reads, batch.n_calls)
    else:
        kmean.pop("pf_k0_load", None)
        kmean.pop("pf_k0_pack", None)
    kernels = {}
    for k, ms in kmean.items():
        b = ab.get(k, 0)
        kernels[k] = {"ms": round(ms, 4), "algo_bytes": int(b),
                      "GBps": round(b / (ms * 1e-3) / 1e9, 2) if ms > 0 else None}
    dom = max(kmean, key=kmean.get)
    achieved = kernels[dom]["GBps"]
    boundary = "records" if record_level else "calls"
    traffic = pmc_traffic(dom, dict(wl, windows_per_gpu=batch.n_windows), boundary)

    # 2. the headline: the rank's whole share, every batch launched every step
    elapsed, total_reads, _, job_outs = timed(dbs)
    value = total_reads / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    job_reads = int(sum(int(o.win_n_reads.sum()) for o in job_outs))
    # every copy of a base window must get the same decision and tags
    dec_by_base = {}
    consistent = True
    for (_, basew), o in zip(groups, job_outs):
        for w, dcs in zip(basew.tolist(), o.decision.tolist()):
            if dec_by_base.setdefault(w, dcs) != dcs:
                consistent = False
    if 0 in range(len(groups)) and groups[0][1].shape[0] == n_base:
        consistent = consistent and all(np.array_equal(o.decision, out.decision) and
                                        np.array_equal(o.read_hp, out.read_hp)
                                        for (_, bw), o in zip(groups, job_outs) if np.array_equal(bw, ident))
    n_probs = 2 * len(share)
    job = {"windows": int(n_job), "tiles": tiles, "base_windows": n_base, "windows_this_gpu": int(len(share)),
           "greedy_problems_this_gpu": int(n_probs), "reads_this_gpu": job_reads,
           "batches_this_gpu": len(dbs), "contexts": split, "copies_consistent": bool(consistent),
           "deal": "weak: a whole job per rank" if args.weak else "LPT on SEQ + MM bytes (pomfret_amd.shard)"}
    if loads is not None:
        job["lpt_loads_max_over_mean"] = round(max(loads) / (sum(loads) / len(loads)), 4)
        job["lpt_bound_ok"] = bool(max(loads) <= lpt_bound(job_costs, world) + 1e-6)
    log(f"[bench] job: {json.dumps(job)}")

    calls_leg = None
    if record_level and not args.no_legs and world == 1:
        # the same reads with K0's calls already resident (the calls-level
        # boundary, pf_batch_upload): K12 + K3 + epilogue only
        dbc = ctx.upload(cfg, batch)
        el_c, tot_c, acc_c, out_c = timed([dbc])
        dbc.free()
        calls_leg = {"value": round(tot_c / el_c, 1), "ms_per_step": round(el_c / args.steps * 1e3, 4),
                     "kernels_ms": {k: round(v / args.steps, 4) for k, v in acc_c.items()
                                    if k not in ("pf_k0_load", "pf_k0_pack")},
                     "decisions_match": bool(np.array_equal(out_c[0].decision, out.decision)),
                     "what": "the first batch's reads, calls resident in HBM (no K0): the pre-K0 boundary"}

    proj = None
    crit = None
    if record_level and not args.no_legs and world == 1 and not args.weak:
        # Strong scaling projected on this GPU: rank 0's LPT share of the same
        # job at N GPUs, timed here (the ranks' shares are equal by the deal:
        # max/mean load below), aggregate = job reads / that step time.
        proj = {}
        for n in (2, 4, 8):
            parts_n = lpt_partition(job_costs, n)
            g_n = split_groups(group_copies(parts_n[0], n_base), min_batches, base_costs)
            extra, dbs_n = [], []
            for gi, (_, basew) in enumerate(g_n):
                hit = next((d for d, (_, bw) in zip(dbs, groups) if np.array_equal(bw, basew)), None)
                if hit is not None and hit not in dbs_n and hit.ctx is ctxs[gi % split]:
                    dbs_n.append(hit)
                else:
                    d, _ = upload(ctxs[gi % split], basew)
                    extra.append(d)
                    dbs_n.append(d)
            el_n, tot_n, _, o_n = timed(dbs_n)
            reads_n = sum(int(o.win_n_reads.sum()) for o in o_n)
            ld = [float(job_costs[p].sum()) for p in parts_n]
            agg = reads_n * n * args.steps / el_n          # every rank runs a share like rank 0's
            proj[str(n)] = {"ms_per_step": round(el_n / args.steps * 1e3, 4), "windows_rank0": int(len(parts_n[0])),
                            "reads_rank0": int(reads_n), "projected_value": round(agg, 1),
                            "projected_speedup": round(agg / value, 3),
                            "lpt_loads_max_over_mean": round(max(ld) / (sum(ld) / n), 4)}
            for d in extra:
                d.free()
            log(f"[bench] strong projection N={n}: {json.dumps(proj[str(n)])}")
        # The same projection over DISTINCT windows: a job of
        # `tiles` contigs with different seeds (a real WGS job has no copies),
        # dealt by LPT on cost estimates (synth_aln.window_cost_estimate: the
        # read bases, replayed from the generator's RNG without building the
        # reads; correlation 0.99998 with the SEQ + MM bytes), then rank 0's
        # share at N=8 generated and timed on this GPU.
        n8 = 8
        td = time.perf_counter()
        djobs = [(replace(spec, seed=seed + 100 + t), w) for t in range(tiles) for w in range(n_base)]
        dcost = window_cost_estimates(djobs, workers=CPU_SHARE)
        parts_d = lpt_partition(dcost, n8)
        ld_d = [float(dcost[p].sum()) for p in parts_d]
        mine = sorted(parts_d[0].tolist())
        a_d = make_aln_batch(spec, jobs=[djobs[i] for i in mine], workers=0)
        dc_d = aln_window_costs(a_d)
        g_d = split_groups([(np.arange(a_d.n_windows), np.arange(a_d.n_windows))], min_batches, dc_d)
        dbs_d = [ctxs[gi % split].upload_aln(cfg, a_d.select(bw) if bw.shape[0] != a_d.n_windows else a_d, lcfg)
                 for gi, (_, bw) in enumerate(g_d)]
        t_gen = time.perf_counter() - td
        el_d, tot_d, _, o_d = timed(dbs_d)
        reads_d = sum(int(o.win_n_reads.sum()) for o in o_d)
        for d in dbs_d:
            d.free()
        del a_d, dbs_d
        proj["8_distinct"] = {
            "ms_per_step": round(el_d / args.steps * 1e3, 4), "windows_rank0": len(mine), "reads_rank0": reads_d,
            "projected_value": round(reads_d * n8 * args.steps / el_d, 1),
            "lpt_loads_max_over_mean": round(max(ld_d) / (sum(ld_d) / n8), 4),
            "job": f"{tiles} contigs x {n_base} windows, seeds {seed + 100}..{seed + 99 + tiles} (no copies)",
            "generate_s": round(t_gen, 1)}
        log(f"[bench] strong projection N=8 distinct: {json.dumps(proj['8_distinct'])}")
        # The floor of a GPU's step: the heaviest base window alone (its
        # serial greedy chain; no GPU count takes it below this)
        wmax = int(np.argmax(out.win_n_reads))
        # both of its problems in pf_k3_heavy, as in the job's batches (alone in
        # a batch the window is its own median: not "heavy" by the rule)
        prev = os.environ.get("PF_K3_HEAVY")
        os.environ["PF_K3_HEAVY"] = "2"
        dbw, _ = upload(ctx, np.array([wmax]))
        if prev is None:
            os.environ.pop("PF_K3_HEAVY")
        else:
            os.environ["PF_K3_HEAVY"] = prev
        el_w, _, acc_w, o_w = timed([dbw])
        dbw.free()
        crit = {"window": wmax, "reads": int(o_w[0].win_n_reads.sum()), "gap_bp": int(gaps[wmax]),
                "ms_per_step": round(el_w / args.steps * 1e3, 4),
                "kernels_ms": {k: round(v / args.steps, 4) for k, v in acc_w.items()},
                "share_of_step_at_8": round(el_w / args.steps * 1e3 / proj["8"]["ms_per_step"], 4)}
        log(f"[bench] critical window: {json.dumps(crit)}")

    fixed_leg = None
    if record_level and not args.no_legs and args.workload == "mix" and world == 1:
        # round 2's headline workload (50 kb gaps, every window decided), one
        # 1024-window batch per context: the rate the gap mix is compared with
        wl50 = dict(WORKLOADS["fixed50"], n_windows=n_base, coverage=wl["coverage"])
        a50 = make_aln_batch(AlnSpec(n_windows=wl50["n_windows"], coverage=wl50["coverage"], gap=wl50["gap"],
                                     seed=seed))
        db50 = ctx.upload_aln(cfg, a50, lcfg)
        el50, tot50, acc50, out50 = timed([db50])
        db50.free()
        out50 = out50[0]
        fixed_leg = {"value": round(tot50 / el50, 1), "ms_per_step": round(el50 / args.steps * 1e3, 4),
                     "reads": int(out50.win_n_reads.sum()), "records": int(a50.n_recs),
                     "kernels_ms": {k: round(v / args.steps, 4) for k, v in acc50.items()},
                     "decisions": {"cis": int((out50.decision == 0).sum()), "trans": int((out50.decision == 1).sum()),
                                   "none": int((out50.decision < 0).sum())},
                     "what": "round 2's workload: 1024 windows x 50 kb gaps at 60x, one batch, records resident"}
        del a50

    # PCIe-inclusive rate (never `value`): the one-shot boundary call hands
    # over host buffers -- upload (validation, pinned staging, H2D), run, D2H
    pcie = None
    if not args.no_legs and record_level:
        t1 = time.perf_counter()
        n_once = 2
        for _ in range(n_once):
            db2 = ctx.upload_aln(cfg, aln0, lcfg)
            db2.run()
            db2.free()
        pcie = {"reads_per_s": round(batch.n_reads * n_once / (time.perf_counter() - t1), 1),
                "ms_per_call": round((time.perf_counter() - t1) / n_once * 1e3, 3),
                "what": "upload(host BAM-record SoA: validation, SEQ repack, H2D) + run + free per call, "
                        "the first batch, rank 0"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and record_level:
        # BASELINE's target is phrased against the reference's -t 32.  The
        # port runs with min(32, effective cores) threads -- the effective
        # cores are the affinity set capped by the cgroup quota (the GPU box
        # grants 16 per GPU) -- over the whole first batch (1024 windows, so
        # the threads are not tail-bound on a few heavy windows), once.  The
        # port parallelises over windows; the reference's kt_for parallelises
        # over contigs (blockjoin.c:4560), which favours the port.  The
        # oracle's results are compared with the GPU's on every window of the
        # batch, and the read tags on the heavy / wide sample.
        eff, eff_how = effective_cores()
        threads = args.cpu_threads or min(32, eff)
        sub = oracle_sample(aln0, gaps, out.win_n_reads)
        n_b0 = int(out.win_n_reads.sum())
        allw = np.arange(aln0.n_windows)
        v_cpu, dt, reps, ref = cpu_baseline_aln(cfg, lcfg, aln0, n_b0, threads, min_cpu_s=0.0, min_reps=1)
        # read tags: the oracle's loader, then its worker (methphase_aln leaves them unset)
        import oracle
        a_sub = aln0.select(sub)
        ref_t = oracle.methphase(cfg, oracle.load_reads(lcfg, a_sub)[0], n_threads=threads)
        bad = sorted(set(compare_with_oracle(out, batch.win_read_off, ref, allw, tags=False))
                     | set(compare_with_oracle(out, batch.win_read_off, ref_t, sub)))
        half = max(1, threads // 2)
        v_half, dt_half = cpu_baseline_aln(cfg, lcfg, aln0, n_b0, half, min_cpu_s=0.0, min_reps=1)[:2]
        eff_scal = v_cpu / (2 * v_half) if v_half else None
        heavy_w = sorted({int(p) >> 1 for p in db.heavy_problems()} & set(sub))
        cpu = {"value": round(v_cpu, 1), "unit": "reads/s", "cores": threads, "kind": "port",
               "sample": f"the whole first batch: {aln0.n_windows} windows, {n_b0} reads, once ({dt:.2f}s wall x "
                         f"{threads} threads); per-window loader + worker over the same BAM records, "
                         f"oracle/pf_oracle{{_load,}}.c; pthreads over windows (the reference's kt_for runs "
                         f"contigs, blockjoin.c:4560)",
               "effective_cores": eff, "effective_cores_from": eff_how,
               "matches": not bad, "mismatched": bad,
               "compared": "every window of the batch: decision, 2x2 tables, join, which_way, score, site/read "
                           f"counts (bit for bit), Fisher p (rtol 1e-6); every read's tag on {len(sub)} windows "
                           "(the 8 with the most reads, the widest gaps >= 400 kb, then the first)",
               "sample_windows": {"n": len(sub), "max_reads": int(out.win_n_reads[sub].max()),
                                  "max_gap_bp": int(gaps[sub].max()), "heavy_problem_windows": len(heavy_w),
                                  "windows_ge_400kb": int((gaps[sub] >= 400_000).sum())},
               "thread_scaling": {str(half): round(v_half, 1), str(threads): round(v_cpu, 1),
                                  "efficiency": round(eff_scal, 3) if eff_scal else None,
                                  "wall_s": {str(half): round(dt_half, 2), str(threads): round(dt, 2)}},
               "t32_linear_estimate": round(v_cpu * 32 / threads, 1),
               "t32_measured": threads == 32 and eff >= 32}
        log(f"[bench] cpu_baseline: {json.dumps(cpu)}")

    # The end-to-end legs time a file-to-output run as a user starts it: the
    # job's resident batches (most of HBM on an 8192-window job) and its host
    # records are released first, so the CLI process and the driver see the
    # device and the page cache a fresh run sees.
    records_per_gpu = (int(sum(int(np.diff(aln.win_rec_off.astype(np.int64))[bw].sum()) for _, bw in groups))
                       if record_level else None)
    n_batches = len(dbs)
    e2e_any = rank == 0 and world == 1 and not args.no_legs and (
        (args.e2e_windows > 0 and record_level) or args.e2e_u_scale > 0)
    if e2e_any:
        for d in dbs:
            d.free()
        dbs = []
        if record_level:
            del aln, aln0, subs, batch
        import gc
        gc.collect()

    e2e = None
    if rank == 0 and world == 1 and not args.no_legs and args.e2e_windows > 0 and record_level:
        threads = args.cpu_threads or min(CPU_SHARE, len(os.sched_getaffinity(0)))
        # (round 2's 64-window BAM: the 50 kb workload, so the fetch rates compare across rounds)
        e2e = e2e_leg(ctx, cfg, lcfg, dict(WORKLOADS["fixed50"], coverage=wl["coverage"]),
                      min(args.e2e_windows, n_base), threads,
                      os.environ.get("TMPDIR", "/tmp"), cpu=not args.no_cpu,
                      cpu_threads=args.cpu_threads or min(32, effective_cores()[0]))
        log(f"[bench] e2e: {json.dumps(e2e)}")

    e2e_u = None
    if rank == 0 and world == 1 and not args.no_legs and args.e2e_u_scale > 0:
        threads = args.cpu_threads or min(CPU_SHARE, len(os.sched_getaffinity(0)))
        e2e_u = e2e_u_leg(ctx, lcfg, threads, os.environ.get("TMPDIR", "/tmp"), scale=args.e2e_u_scale,
                          cpu=not args.no_cpu, cpu_threads=args.cpu_threads or min(32, effective_cores()[0]))
        log(f"[bench] e2e_u: {json.dumps(e2e_u)}")
        if e2e_u.get("k4"):
            kernels[e2e_u["k4"]["kernel"]] = {"ms": e2e_u["k4"]["ms"], "algo_bytes": e2e_u["k4"]["algo_bytes"],
                                              "GBps": e2e_u["k4"]["GBps"], "leg": "e2e_u (largest contig)"}

    par = (f"job windows dealt over dp{world} by LPT (strong)" if not args.weak
           else f"dp{world}, a whole job per rank (weak)")
    res = {
        "metric": "aligned reads/sec (methphase kernel)",
        "value": round(value, 1),
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": "u32/f32",
        "data": f"synthetic (seeded {wl['coverage']}x long-read pileups, HG002-like; HG002 not available offline)",
        "config": {
            "workload": (f"HG002-like WGS-sized job at {wl['coverage']}x, pre-haplotagged: {n_job} gap windows = "
                         + (f"{tiles} copies of {n_base} distinct windows (" if tiles > 1 else f"{n_base} distinct windows (")
                         + ("gaps log-uniform 5-500 kb (SURVEY 8d mix), "
                            f"{wl['skip_frac']:.0%} skipped (left tags lost) + {wl['nosite_frac']:.0%} site-less "
                            "windows" if wl["gap_mix"] else f"gaps {wl['gap'] // 1000} kb")
                         + f"); {len(share)} windows on this GPU"
                         + (" (a whole job per rank)" if args.weak else "")
                         + "; " + ("BAM records resident (every per-batch kernel in the step: K0 loader, scan + "
                                   "pack, K12, K2, K3)" if record_level else "reads + 5mC calls resident (no K0)")),
            "boundary": boundary,
            "windows_job": n_job, "windows_per_gpu": int(len(share)),
            "records_per_gpu": records_per_gpu,
            "reads_per_gpu": job_reads, "coverage": wl["coverage"],
            "cov_for_selection": cfg.cov_for_selection, "cov_for_runtime": cfg.cov_for_runtime,
            "n_cand": cfg.n_cand, "k": cfg.k, "k_span": cfg.k_span,
            "parallelism": par,
            "batches_per_gpu": n_batches, "contexts_per_gpu": split,
        },
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": PEAK_HBM_GBPS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBPS, 5) if achieved else None,
                     "traffic": traffic, "measured_on": "single_batch"},
        "kernels": kernels,
        "cpu_baseline": cpu,
        "vs_cpu_baseline": round(value / cpu["value"], 2) if cpu else None,
        "vs_cpu_t32_estimate": round(value / cpu["t32_linear_estimate"], 2) if cpu else None,
        "job": job,
        "single_batch": single,
        "strong_projection": proj,
        "critical_window": crit,
        "pcie_inclusive": pcie,
        "e2e": e2e,
        "e2e_u": e2e_u,
        "calls_level": calls_leg,
        "fixed_gap50": fixed_leg,
        "decisions": {"cis": int((out.decision == 0).sum()), "trans": int((out.decision == 1).sum()),
                      "none": int((out.decision < 0).sum()), "of": "the first batch"},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    for d in dbs:
        d.free()
    for c in ctxs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
