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
The batch's windows run as `--split` (default 2) batches on as many contexts
of the GPU, launched together every step -- what the driver does with its
PF_DEV_CONTEXTS contexts per GPU; the single-batch run of the same step is
timed too and gives the per-kernel figures and the roofline.
`--calls-level` times the previous boundary instead (reads and 5mC calls
resident, no K0).  Workload at N=1: BASELINE.json's target is quoted on HG002
60x at 1 GPU, so the job is 1024 gap windows of 50 kb at 60x (HG002-like,
synthesised -- HG002 is not available offline), parameters as `pomfret
methphase` derives them without -c (cov_for_selection 7, cov_for_runtime 14,
n_cand 16; blockjoin.c:4373-4375), loader defaults -q 10 -L 15000, ML bands
100/156 (cli.c:52-63).  --coverage 30 --windows 256 is configs[1]'s shape.

Multi-GPU (torchrun, one process per GPU): weak scaling by default -- the
path partitions into independent windows, and a real run (a whole genome:
tens of thousands of windows) keeps every GPU's share large as N grows, so
every rank owns a batch of --windows windows of its own (seeds differ per
rank); no collective in the data path; after each step the int8 decisions
are gathered to every rank over RCCL (the drop-in's only exchange: the host
that writes VCF/GTF needs all decisions).  --strong deals one job's windows
over the ranks instead (total work fixed).

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


def cpu_baseline_aln(cfg, lcfg, aln, n_reads, threads: int, min_cpu_s: float = 20.0, max_reps: int = 200):
    """Record-level CPU path of the oracle (per window: loader + worker, the
    reference's structure), `threads` pthreads over windows, bounded sample."""
    import oracle
    t0 = time.perf_counter()
    reps = 0
    while reps < max_reps:
        oracle.methphase_aln(cfg, lcfg, aln, n_threads=threads)
        reps += 1
        if (time.perf_counter() - t0) * threads >= min_cpu_s and reps >= 2:
            break
    dt = time.perf_counter() - t0
    return n_reads * reps / dt, dt, reps


def e2e_leg(ctx, cfg, lcfg, wl, n_windows: int, threads: int, workdir: str, cpu: bool = True):
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
                    `threads` threads (the reference's structure: htslib decode
                    + the kt_for worker)."""
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
            # (estimate_read_coverage_dirtyfast): device fetch vs the serial host pass
            c0 = time.perf_counter()
            cov_d = b.estimate_coverage_device(ctx)
            c1 = time.perf_counter()
            cov_h = b.estimate_coverage()
            c2 = time.perf_counter()
            res["coverage_estimate"] = {"device_ms": round((c1 - c0) * 1e3, 1), "host_ms": round((c2 - c1) * 1e3, 1),
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
                t3 = time.perf_counter()
                ref = oracle.methphase_aln(cfg, lcfg, got, n_threads=threads)
                t4 = time.perf_counter()
                res["cpu_port"] = {"reads_per_s": round(reads / ((t1 - t0) + (t4 - t3)), 1),
                                   "ms": round(((t1 - t0) + (t4 - t3)) * 1e3, 1),
                                   "what": f"host fetch ({threads} threads) + oracle record-level worker "
                                           f"({threads} threads)"}
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


def e2e_u_leg(ctx, lcfg, threads: int, workdir: str, scale: float = 1.0, cpu: bool = True):
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
      cpu_port: the product's planner / writers with the host reader, the
                serial host coverage pass and the oracle computing every job
                (tests/_oracle_pipeline.methphase_files_port, `threads`
                threads);
    outputs compared byte for byte.  Also the K4 kernel on the largest
    contig's reads (HIP events, SURVEY 8d's -u bytes)."""
    import subprocess
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import _genome
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
                                          threads=threads)
            outs["cpu_port"] = take(prefix + ".port")
            res["cpu_port"] = {"s": round(ph["total_s"], 2), "records_per_s": round(res["records"] / ph["total_s"], 1),
                               "phases_s": {k: round(v, 2) for k, v in ph.items() if k != "total_s"},
                               "what": f"host reader + serial host coverage pass + oracle jobs, {threads} threads"}
            res["vs_cpu_port"] = round(ph["total_s"] / (t1 - t0), 2)
        res["outputs_identical"] = all(o == outs["cli"] for o in outs.values())
        res["compared"] = sorted(outs)
    finally:
        for f in (g["bam"], g["bam"] + ".bai", g["vcf"]):
            if os.path.exists(f):
                os.unlink(f)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--windows", type=int, default=WORKLOAD["n_windows"],
                    help="windows per rank (weak scaling, the default); the job's windows with --strong")
    ap.add_argument("--coverage", type=int, default=WORKLOAD["coverage"])
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="mix",
                    help="mix: log-uniform 5-500 kb gaps with skipped / site-less windows; fixed50: 50 kb gaps")
    ap.add_argument("--weak", action="store_true", help="every rank owns --windows windows of its own (default)")
    ap.add_argument("--strong", action="store_true", help="one job of --windows windows dealt over the ranks")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-legs", action="store_true", help="skip the calls-level and PCIe-inclusive legs")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--e2e-windows", type=int, default=64,
                    help="windows of the end-to-end (BAM file -> decisions) leg; 0 skips it")
    ap.add_argument("--e2e-u-scale", type=float, default=1.0,
                    help="genome scale of the configs[3]-shaped -u leg (1.0: 96 Mb, ~1,000 windows); 0 skips it")
    ap.add_argument("--split", type=int, default=2,
                    help="the windows as this many batches on as many contexts of the GPU, launched together "
                         "(the headline; the single-batch run is kept for the per-kernel figures); 1: one batch")
    ap.add_argument("--calls-level", action="store_true",
                    help="time the calls-level boundary (reads + 5mC calls resident, no K0)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from pomfret_amd import Config, Context, LoadConfig, WindowBatch
    from pomfret_amd.synth import SynthSpec, make_batch
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch

    args.weak = not args.strong
    wl = dict(WORKLOADS[args.workload], n_windows=args.windows, coverage=args.coverage)
    cfg = Config.from_coverage(wl["coverage"], given=False)
    lcfg = LoadConfig()
    record_level = not args.calls_level
    # Weak scaling (default): every rank owns wl["n_windows"] windows of its
    # own.  --strong: one job of wl["n_windows"] windows, dealt round-robin to
    # the ranks (the synthetic windows are i.i.d.; the product's sharder,
    # pomfret_amd.shard, balances real windows by LPT on their bytes).
    if args.weak:
        mine = list(range(wl["n_windows"]))
        seed = 1000 + rank
    else:
        mine = list(range(rank, wl["n_windows"], world))
        seed = 1000
    t = time.perf_counter()
    if record_level:
        # generated (in worker processes) before anything touches the GPU
        aln = make_aln_batch(AlnSpec(n_windows=wl["n_windows"], coverage=wl["coverage"], gap=wl["gap"], seed=seed,
                                     gap_mix=wl["gap_mix"], skip_frac=wl["skip_frac"],
                                     nosite_frac=wl["nosite_frac"]),
                             windows=mine, workers=0 if world == 1 else max(1, CPU_SHARE // 2))
        log(f"[bench] rank {rank}: generated {aln.n_windows} windows, {aln.n_recs} BAM records "
            f"({aln.nbytes() / 1e9:.2f} GB) in {time.perf_counter() - t:.1f}s")

    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend="nccl")
        dist = tdist
    ctx = Context(local_rank)
    if record_level:
        t = time.perf_counter()
        db = ctx.upload_aln(cfg, aln, lcfg)
        log(f"[bench] upload (validation, SEQ repack, H2D; no device work): {time.perf_counter() - t:.1f}s")
        off, cpos, ccat, _, _ = db.debug_calls()
        rr = db.read_recs()
        # the loaded reads as a window batch (the byte model and the calls-level
        # leg): K0's calls, and the spans of the kept records (pos, bam_endpos)
        wro = np.searchsorted(rr, aln.win_rec_off.astype(np.int64)).astype(np.uint32)
        rs, re_ = record_spans(aln, rr)
        batch = WindowBatch(win_start=aln.win_start, win_end=aln.win_end, win_read_off=wro,
                            read_start=rs, read_end=re_,
                            read_hp=aln.hp[rr], read_call_off=off, call_pos=cpos, call_cat=ccat,
                            win_cov_sel=aln.win_cov_sel, win_cov_rt=aln.win_cov_rt, win_n_cand=aln.win_n_cand)
        del off, cpos, ccat
    else:
        batch = make_batch(SynthSpec(n_windows=wl["n_windows"], coverage=wl["coverage"], gap=wl["gap"],
                                     seed=seed)).select(mine)
        log(f"[bench] rank {rank}: generated {batch.n_windows} windows, {batch.n_reads} reads, "
            f"{batch.n_calls} calls in {time.perf_counter() - t:.1f}s")
        db = ctx.upload(cfg, batch)

    def timed(dbs, n_windows, n_reads, parts=None):
        """W warmup runs, then exactly K timed steps between barrier + sync
        pairs; returns (max-over-ranks seconds, total reads, per-kernel ms
        summed over the steps, one step's result).  dbs: one batch, or the
        batch's windows as several batches (parts: their window indices), each
        on its own context, launched together every step."""
        if not isinstance(dbs, (list, tuple)):
            dbs = [dbs]
        outs = [[d.run(), d.run()] for d in dbs]
        for _ in range(args.warmup):
            for d, o in zip(dbs, outs):
                d.run(o[0])
        if dist is not None:
            import torch
            n_max = torch.tensor([n_windows], dtype=torch.int64, device=f"cuda:{local_rank}")
            dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
            dec_t = torch.full((int(n_max.item()),), -2, dtype=torch.int8, device=f"cuda:{local_rank}")
            gathered = torch.empty(world * dec_t.numel(), dtype=torch.int8, device=f"cuda:{local_rank}")

        def merged(k):
            if len(dbs) == 1:
                return outs[0][k % 2].decision
            dec = np.empty(n_windows, dtype=np.int8)
            for p, o in zip(parts, outs):
                dec[p] = o[k % 2].decision
            return dec

        # Steps are pipelined two deep (pf_methphase_launch / _finish): the host
        # epilogue of step k (Fisher tests, decisions, read tags) overlaps the
        # kernels of step k+1; every step runs every kernel (K0 loader, scan +
        # pack, K12, K2, K3), the D2H copy and the epilogue inside the timed region.
        def finish(k):
            for d, o in zip(dbs, outs):
                d.finish(o[k % 2])
            if dist is not None:
                dec_t[:n_windows].copy_(torch.from_numpy(merged(k)))
                dist.all_gather_into_tensor(gathered, dec_t)

        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        kern_acc = {}
        if args.steps:
            for d in dbs:
                d.launch()
        for k in range(args.steps):
            if k + 1 < args.steps:
                for d in dbs:
                    d.launch()
            finish(k)
            for d in dbs:
                for kn, v in d.ctx.kernel_times().items():
                    kern_acc[kn] = kern_acc.get(kn, 0.0) + v
        if dist is not None:
            torch.cuda.synchronize()
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
            rt = torch.tensor([n_reads], dtype=torch.float64, device=f"cuda:{local_rank}")
            dist.all_reduce(rt)
            total = float(rt.item()) * args.steps
        else:
            total = float(n_reads) * args.steps
        out = outs[0][(args.steps - 1) % 2]
        if len(dbs) > 1:
            out = {"decision": merged(args.steps - 1)}
        return elapsed, total, kern_acc, out

    elapsed, total_reads, kern_acc, out = timed(db, batch.n_windows, batch.n_reads)
    value = total_reads / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    stats = db.stats()
    kmean = {k: v / args.steps for k, v in kern_acc.items()}
    ab = algo_bytes(batch, stats, out.win_n_sites, db.heavy_problems())
    if record_level:
        ab["pf_k0_load"] = k0_bytes(aln, rr, batch.n_calls)
        ab["pf_k0_pack"] = pack_bytes(aln.n_recs, batch.n_reads, batch.n_calls)
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

    calls_leg = None
    if record_level and not args.no_legs:
        # the same reads with K0's calls already resident (the calls-level
        # boundary, pf_batch_upload): K12 + K3 + epilogue only
        dbc = ctx.upload(cfg, batch)
        el_c, tot_c, acc_c, out_c = timed(dbc, batch.n_windows, batch.n_reads)
        dbc.free()
        calls_leg = {"value": round(tot_c / el_c, 1), "ms_per_step": round(el_c / args.steps * 1e3, 4),
                     "kernels_ms": {k: round(v / args.steps, 4) for k, v in acc_c.items()
                                    if k not in ("pf_k0_load", "pf_k0_pack")},
                     "decisions_match": bool(np.array_equal(out_c.decision, out.decision)),
                     "what": "same reads, calls resident in HBM (no K0): the pre-K0 boundary"}

    fixed_leg = None
    if record_level and not args.no_legs and args.workload == "mix" and world == 1:
        # round 2's headline workload (50 kb gaps, every window decided), same
        # steps: the rate the gap mix is compared with
        wl50 = dict(WORKLOADS["fixed50"], n_windows=wl["n_windows"], coverage=wl["coverage"])
        a50 = make_aln_batch(AlnSpec(n_windows=wl50["n_windows"], coverage=wl50["coverage"], gap=wl50["gap"],
                                     seed=seed), windows=mine)
        db50 = ctx.upload_aln(cfg, a50, lcfg)
        nr50 = int(db50.run().win_n_reads.sum())
        el50, tot50, acc50, out50 = timed(db50, a50.n_windows, nr50)
        db50.free()
        fixed_leg = {"value": round(tot50 / el50, 1), "ms_per_step": round(el50 / args.steps * 1e3, 4),
                     "reads": nr50, "records": int(a50.n_recs),
                     "kernels_ms": {k: round(v / args.steps, 4) for k, v in acc50.items()},
                     "decisions": {"cis": int((out50.decision == 0).sum()), "trans": int((out50.decision == 1).sum()),
                                   "none": int((out50.decision < 0).sum())},
                     "what": "round 2's workload: 1024 windows x 50 kb gaps at 60x, records resident"}
        del a50

    split_leg = None
    if record_level and args.split > 1:
        # the same windows as S batches, each on its own context of this GPU
        # (own streams, own device buffers), launched together every step: one
        # batch's K0/K12 fill the CUs the other's K3 tail leaves idle.  Windows
        # are dealt to the batches heaviest first (record counts), round-robin.
        nrec_w = np.diff(aln.win_rec_off.astype(np.int64))
        order = np.argsort(-nrec_w, kind="stable")
        parts = [sorted(order[s::args.split].tolist()) for s in range(args.split)]
        sctx = [ctx] + [Context(local_rank) for _ in range(args.split - 1)]
        sdb = [c.upload_aln(cfg, aln.select(p), lcfg) for c, p in zip(sctx, parts)]
        el_s, tot_s, _, out_s = timed(sdb, batch.n_windows, batch.n_reads, [np.asarray(p) for p in parts])
        split_leg = {"value": round(tot_s / el_s, 1), "ms_per_step": round(el_s / args.steps * 1e3, 4),
                     "batches": args.split,
                     "decisions_match": bool(np.array_equal(out_s["decision"], out.decision)),
                     "what": f"same windows as {args.split} batches on {args.split} contexts of this GPU "
                             "(windows dealt heaviest first), launched together every step"}
        log(f"[bench] split: {json.dumps(split_leg)}")
        for d in sdb:
            d.free()
        for c in sctx[1:]:
            c.close()

    # PCIe-inclusive rate (never `value`): the one-shot boundary call hands
    # over host buffers -- upload (validation, pinned staging, H2D), run, D2H
    pcie = None
    if not args.no_legs:
        t1 = time.perf_counter()
        n_once = 2
        for _ in range(n_once):
            db2 = ctx.upload_aln(cfg, aln, lcfg) if record_level else ctx.upload(cfg, batch)
            db2.run()
            db2.free()
        what = ("upload(host BAM-record SoA: validation, SEQ repack, H2D) + run + free per call"
                if record_level else "upload(host SoA -> HBM) + run + free per call")
        pcie = {"reads_per_s": round(batch.n_reads * n_once / (time.perf_counter() - t1), 1),
                "ms_per_call": round((time.perf_counter() - t1) / n_once * 1e3, 3),
                "what": what + ", rank 0"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # the box's CPU share per GPU (OMP_NUM_THREADS there); the reference's
        # kt_for scales with threads, so the -t 32 figure of BASELINE's target
        # would be at most twice this
        # BASELINE's target is phrased against the reference's -t 32: 32
        # threads when this host's affinity allows it (the GPU box's share is
        # 16 cores per GPU: the 16-thread rate is reported beside it)
        threads = args.cpu_threads or min(32, len(os.sched_getaffinity(0)))
        sub = list(range(min(64, batch.n_windows)))
        if record_level:
            a_sub = aln.select(sub)
            n_sub = int(batch.win_read_off[len(sub)])
            v_cpu, dt, reps = cpu_baseline_aln(cfg, lcfg, a_sub, n_sub, threads, min_cpu_s=30.0)
            # thread scaling of the same sample (windows are independent; the
            # reference's -t N is kt_for over contigs)
            v_half = cpu_baseline_aln(cfg, lcfg, a_sub, n_sub, max(1, threads // 2), min_cpu_s=15.0)[0]
            what = "per-window loader + worker over the same BAM records, oracle/pf_oracle{_load,}.c"
        else:
            b_sub = batch.select(sub)
            n_sub = b_sub.n_reads
            v_cpu, dt, reps = cpu_baseline(cfg, b_sub, threads)
            v_half = cpu_baseline(cfg, b_sub, max(1, threads // 2), min_cpu_s=10.0)[0]
            what = "oracle/pf_oracle.c"
        eff = v_cpu / (2 * v_half) if v_half else None
        cpu = {"value": round(v_cpu, 1), "unit": "reads/s", "cores": threads, "kind": "port",
               "sample": f"the first {len(sub)} windows of the workload x{reps} "
                         f"({n_sub * reps} reads, {dt:.2f}s wall x {threads} threads "
                         f"= {dt * threads:.0f} CPU-s), {what}; {threads} threads "
                         f"({len(os.sched_getaffinity(0))} in this process's affinity; the box's share per GPU "
                         f"is {CPU_SHARE})",
               "thread_scaling": {str(max(1, threads // 2)): round(v_half, 1), str(threads): round(v_cpu, 1),
                                  "efficiency": round(eff, 3) if eff else None},
               "t32_linear_estimate": round(v_cpu * 32 / threads, 1), "t32_measured": threads == 32}

    e2e = None
    if rank == 0 and world == 1 and not args.no_legs and args.e2e_windows > 0:
        threads = args.cpu_threads or min(CPU_SHARE, len(os.sched_getaffinity(0)))
        # (round 2's 64-window BAM: the 50 kb workload, so the fetch rates compare across rounds)
        e2e = e2e_leg(ctx, cfg, lcfg, dict(WORKLOADS["fixed50"], coverage=wl["coverage"]),
                      min(args.e2e_windows, wl["n_windows"]), threads,
                      os.environ.get("TMPDIR", "/tmp"), cpu=not args.no_cpu)
        log(f"[bench] e2e: {json.dumps(e2e)}")

    e2e_u = None
    if rank == 0 and world == 1 and not args.no_legs and args.e2e_u_scale > 0:
        threads = args.cpu_threads or min(CPU_SHARE, len(os.sched_getaffinity(0)))
        e2e_u = e2e_u_leg(ctx, lcfg, threads, os.environ.get("TMPDIR", "/tmp"), scale=args.e2e_u_scale,
                          cpu=not args.no_cpu)
        log(f"[bench] e2e_u: {json.dumps(e2e_u)}")
        if e2e_u.get("k4"):
            kernels[e2e_u["k4"]["kernel"]] = {"ms": e2e_u["k4"]["ms"], "algo_bytes": e2e_u["k4"]["algo_bytes"],
                                              "GBps": e2e_u["k4"]["GBps"], "leg": "e2e_u (largest contig)"}

    single = None
    if split_leg is not None:
        # the headline is the split run (the driver's default: PF_DEV_CONTEXTS
        # contexts per GPU); the per-kernel figures and the roofline come from
        # the single-batch run, where each kernel runs alone on the GPU
        single = {"value": round(value, 1), "ms_per_step": round(ms_per_step, 4),
                  "what": "the windows as one batch on one context (kernels and roofline measured here)"}
        value = split_leg["value"]
        ms_per_step = split_leg["ms_per_step"]
    par = f"windows dealt over dp{world}" + (" (weak: per-rank batches)" if args.weak else " (strong: one job)")
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
            "workload": (f"HG002-like {wl['coverage']}x pre-haplotagged: "
                         f"{wl['n_windows'] * (world if args.weak else 1)} gap windows, "
                         + ("gaps log-uniform 5-500 kb (SURVEY 8d mix), "
                            f"{wl['skip_frac']:.0%} skipped (left tags lost) + {wl['nosite_frac']:.0%} site-less windows "
                            if wl["gap_mix"] else f"gaps {wl['gap'] // 1000} kb ")
                         + f"in the job, {batch.n_windows} on this GPU; "
                         + ("BAM records resident (every per-batch kernel in the step: K0 loader, scan + pack, "
                            "K12, K2, K3)" if record_level else "reads + 5mC calls resident (no K0)")),
            "boundary": boundary,
            "records_per_gpu": aln.n_recs if record_level else None,
            "windows_per_gpu": batch.n_windows, "reads_per_gpu": batch.n_reads,
            "calls_per_gpu": batch.n_calls, "coverage": wl["coverage"],
            "cov_for_selection": cfg.cov_for_selection, "cov_for_runtime": cfg.cov_for_runtime,
            "n_cand": cfg.n_cand, "k": cfg.k, "k_span": cfg.k_span,
            "parallelism": par,
            "batches_per_gpu": args.split,
        },
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": PEAK_HBM_GBPS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBPS, 5) if achieved else None,
                     "traffic": traffic},
        "kernels": kernels,
        "cpu_baseline": cpu,
        "vs_cpu_baseline": round(value / cpu["value"], 2) if cpu else None,
        # BASELINE's target is phrased against the reference's -t 32: the
        # 16-thread port scaled linearly to 32 threads (an upper bound for it)
        "vs_cpu_t32_estimate": round(value / cpu["t32_linear_estimate"], 2) if cpu else None,
        "pcie_inclusive": pcie,
        "e2e": e2e,
        "e2e_u": e2e_u,
        "calls_level": calls_leg,
        "fixed_gap50": fixed_leg,
        "split": split_leg,
        "single_batch": single,
        "decisions": {"cis": int((out.decision == 0).sum()), "trans": int((out.decision == 1).sum()),
                      "none": int((out.decision < 0).sum())},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    db.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
