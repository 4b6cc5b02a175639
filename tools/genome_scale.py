"""Genome-scale `methphase -u` when the -u arenas overflow the device
(VERDICT r05 "next round" 2), and an HG002 60x wall-clock projection that
prices it.

The -u pre-pass inflates every contig once and keeps the inflated arenas in
HBM for the window jobs (pf_ingest.hip ArenaCache).  HG002 at 60x is ~194 GB
of BAM and ~310 GB inflated: more than one MI355X holds, so on one GPU the
window jobs of the contigs past the budget read and inflate their BAM again
(blockjoin.c's worker 4350-4426 reads each window's records from the file;
the pre-pass is 1841-1898).  On the 96 Mb 4-contig genome of bench.py's e2e_u
leg this measures, with outputs compared byte for byte:
  keep      the default (every arena kept: 4 hits);
  budget    PF_ARENA_KEEP_MAX set to about half the inflated genome (the
            contigs past it miss and are re-read);
  no_cache  PF_FETCH_CACHE=0 (every window job re-reads);
each as the CLI a user runs (wall clock) and as the in-process driver (its
pf_mp_stats: arena hits, misses, re-read bytes, per-phase seconds); the CPU
port once for the outputs.  It also times an O_DIRECT read of the BAM (the
box's storage without the page cache), the bandwidth a BAM too large for the
page cache is read at.

Then the PROJECTION (not a measurement) for 1 and 8 GPUs: per-Mb phase rates
from the runs above, the kept fraction from the arena budget per GPU (HBM
minus the keep rule's reserve, pf_ingest.hip), misses priced at the measured
no-cache window rate, and the BAM reads priced at the page-cache rate the runs
saw and at the measured O_DIRECT rate (the node's storage is shared by its 8
GPUs).

usage: python tools/genome_scale.py [--no-cpu] > profiles/r06/genome_scale.json
       python tools/genome_scale.py --project saved.json   (the projection again)"""
import json
import mmap
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))

import _genome  # noqa: E402
from bench import effective_cores  # noqa: E402
from pomfret_amd import Context, LoadConfig  # noqa: E402
from pomfret_amd.pipeline import methphase_files  # noqa: E402

HG002_MB = 3_100            # GRCh38 primary assembly (Mb)
HBM_BYTES = 288e9           # one MI355X


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def odirect_read_gbps(path, limit=8 << 30):
    """GB/s of an O_DIRECT sequential read of `path` (1 GiB requests), or an
    error string (tmpfs and some filesystems refuse O_DIRECT)."""
    try:
        fd = os.open(path, os.O_RDONLY | os.O_DIRECT)
    except OSError as e:
        return f"unavailable: {e}"
    buf = mmap.mmap(-1, 1 << 30)
    n = 0
    t = time.perf_counter()
    try:
        while n < limit:
            k = os.readv(fd, [buf])
            if k <= 0:
                break
            n += k
    except OSError as e:
        return f"unavailable: {e}"
    finally:
        os.close(fd)
        buf.close()
    dt = time.perf_counter() - t
    return round(n / dt / 1e9, 2) if n else "unavailable: read nothing"


def hbm_total_bytes(out=None):
    if out and out.get("hbm_total_bytes"):
        return int(out["hbm_total_bytes"])
    try:
        import torch
        return int(torch.cuda.get_device_properties(0).total_memory)
    except Exception:  # noqa: BLE001
        return int(HBM_BYTES)


def main():
    if "--project" in sys.argv:            # recompute the projection of a saved run
        out = json.load(open(sys.argv[sys.argv.index("--project") + 1]))
        out["hg002_60x_projection"] = project(out, out["genome"]["genome_mb"])
        print(json.dumps(out), flush=True)
        return
    cpu = "--no-cpu" not in sys.argv
    eff, _ = effective_cores()
    threads = min(16, eff)
    workdir = os.environ.get("TMPDIR", "/tmp")
    spec = _genome.GenomeSpec()
    prefix = os.path.join(workdir, f"pf_gs_{os.getpid()}")
    t = time.perf_counter()
    g = _genome.write_genome(prefix, spec, workers=threads)
    mb = sum(L for _, L in spec.contigs) / 1e6
    out = {"what": "methphase -u, no -c, 60x, the 96 Mb 4-contig genome of bench.py's e2e_u leg, with the kept "
                   "-u arenas capped (PF_ARENA_KEEP_MAX) or off (PF_FETCH_CACHE=0)",
           "genome": {"contigs": [[n, L] for n, L in spec.contigs], "genome_mb": mb, "records": g["n_records"],
                      "bam_bytes": g["bam_bytes"], "gen_s": round(time.perf_counter() - t, 1)},
           "threads": threads}
    log(f"[gs] generated {g['n_records']} records, {g['bam_bytes'] / 2**30:.2f} GiB")
    ctx = Context(0)
    outs = {}

    def take(pre):
        o = [open(pre + e, "rb").read() for e in (".mp.vcf", ".mp.gtf")]
        for e in (".mp.vcf", ".mp.gtf"):
            os.unlink(pre + e)
        return o

    try:
        out["odirect_read_gbps"] = odirect_read_gbps(g["bam"])
        log(f"[gs] O_DIRECT read: {out['odirect_read_gbps']}")
        # the inflated genome, from a default run's pre-pass
        runs = {}
        modes = [("keep", {}), ("budget", None), ("no_cache", {"PF_FETCH_CACHE": "0"})]
        for name, env in modes:
            if env is None:       # about half the inflated genome: some contigs keep, the rest miss
                infl = runs["keep"]["driver"]["phases"]["haptag"]["inflated_bytes"]
                env = {"PF_ARENA_KEEP_MAX": str(int(infl * 0.5))}
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                cli = os.path.join(HERE, "pomfret_amd", "pomfret-amd")
                cmd = [cli, "methphase", "-u", "-v", "-t", str(threads), "-o", prefix + f".{name}.cli", "--vcf",
                       g["vcf"], g["bam"]]
                t0 = time.perf_counter()
                p = subprocess.run(cmd, capture_output=True, text=True)
                dt = time.perf_counter() - t0
                if p.returncode != 0:
                    raise RuntimeError(f"pomfret-amd failed ({p.returncode}): {p.stderr[-2000:]}")
                outs[f"{name}.cli"] = take(prefix + f".{name}.cli")
                t0 = time.perf_counter()
                r = methphase_files(g["bam"], g["vcf"], prefix + f".{name}.drv", None, LoadConfig(), ctx=ctx,
                                    untagged=True, threads=threads)
                dd = time.perf_counter() - t0
                outs[f"{name}.driver"] = take(prefix + f".{name}.drv")
                st = r["stats"]
                runs[name] = {"env": env, "cli_s": round(dt, 3),
                              "cli_phases": [ln for ln in p.stderr.splitlines() if "phases:" in ln],
                              "driver": {"s": round(dd, 3), "arena_hits": st["arena_hits"],
                                         "arena_misses": st["arena_misses"], "reread_bytes": st["reread_bytes"],
                                         "phases": st}}
                log(f"[gs] {name}: cli {dt:.2f}s driver {dd:.2f}s hits {st['arena_hits']} misses "
                    f"{st['arena_misses']} reread {st['reread_bytes'] / 2**30:.2f} GiB")
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        out["runs"] = runs
        if cpu:
            from _oracle_pipeline import methphase_files_port
            rp, ph = methphase_files_port(g["bam"], g["vcf"], prefix + ".port", None, LoadConfig(), untagged=True,
                                          threads=min(32, eff))
            outs["cpu_port"] = take(prefix + ".port")
            out["cpu_port"] = {"s": round(ph["total_s"], 2), "threads": min(32, eff)}
        first = outs["keep.cli"]
        out["outputs_identical"] = all(o == first for o in outs.values())
        out["compared"] = sorted(outs)
    finally:
        for f in (g["bam"], g["bam"] + ".bai", g["vcf"]):
            if os.path.exists(f):
                os.unlink(f)
        ctx.close()
    out["hg002_60x_projection"] = project(out, mb)
    print(json.dumps(out), flush=True)


def project(out, mb):
    """Wall clock of HG002 60x on 1 and 8 GPUs from the per-Mb rates above."""
    R = out["runs"]
    keep, nc = R["keep"]["driver"]["phases"], R["no_cache"]["driver"]["phases"]
    gb = out["genome"]["bam_bytes"]
    infl = keep["haptag"]["inflated_bytes"]
    per_mb = lambda x: x / mb                                     # noqa: E731
    bam_mb, infl_mb = per_mb(gb), per_mb(infl)
    t_plan = per_mb(keep["s_plan"] + keep["s_estimate"])
    t_pre = per_mb(keep["s_haptag"])                             # read + inflate + K4, page-cache fed
    t_win_hit = per_mb(keep["s_windows"])
    t_win_miss = per_mb(nc["s_windows"])                          # every window job re-reads and inflates
    t_fin = per_mb(keep["s_finish"])
    read_ms = keep["haptag"]["read_ms"]
    pc_gbps = keep["haptag"]["comp_bytes"] / (read_ms / 1e3) / 1e9 if read_ms else None
    hbm = hbm_total_bytes(out)
    out["hbm_total_bytes"] = hbm
    budget = hbm - max(hbm / 3, 32 * 2**30)                       # pf_ingest.hip's keep rule leaves this free
    od = out["odirect_read_gbps"] if isinstance(out["odirect_read_gbps"], float) else None
    res = {"kind": "PROJECTION from the per-Mb rates measured above, not a measurement",
           "genome_mb": HG002_MB, "bam_gb": round(bam_mb * HG002_MB / 1e9, 1),
           "inflated_gb": round(infl_mb * HG002_MB / 1e9, 1),
           "arena_budget_gb_per_gpu": round(budget / 1e9, 1),
           "page_cache_read_gbps_measured": round(pc_gbps, 2) if pc_gbps else None,
           "odirect_read_gbps_measured": od,
           "per_mb_s": {"plan": round(t_plan, 6), "prepass": round(t_pre, 6), "windows_hit": round(t_win_hit, 6),
                        "windows_miss": round(t_win_miss, 6), "writers": round(t_fin, 6)}}
    for n in (1, 8):
        share = HG002_MB / n
        kept = min(1.0, budget / (infl_mb * share)) if infl_mb else 1.0     # infl_mb: bytes per Mb
        win = share * (kept * t_win_hit + (1 - kept) * t_win_miss)
        pre = share * t_pre
        t_pc = HG002_MB * t_plan + pre + win + HG002_MB * t_fin
        e = {"kept_fraction": round(kept, 3), "prepass_s": round(pre, 1), "windows_s": round(win, 1),
             "page_cache_fed_s": round(t_pc, 1)}
        if od:
            # the node's storage, shared by its GPUs: the whole BAM once (pre-pass)
            # plus the missed contigs' re-reads, at the O_DIRECT rate
            read_s = (bam_mb * HG002_MB * (1 + (1 - kept))) / (od * 1e9)
            e["storage_read_s"] = round(read_s, 1)
            e["storage_fed_s"] = round(max(t_pc, read_s + HG002_MB * (t_plan + t_fin)), 1)
        res[f"{n}_gpu"] = e
    res["assumes"] = ("HG002-like density as the synthetic genome (60x, 1 het SNV per kb, phase gaps every "
                      "50-100 kb); contigs dealt evenly over the GPUs; the pre-pass re-inflates nothing; a miss "
                      "costs the no-cache run's per-Mb window time; the writers' rescue fetches as measured; "
                      "storage-fed: the BAM cannot stay in the page cache, so every read runs at the O_DIRECT rate "
                      "and the GPUs wait for it")
    return res


if __name__ == "__main__":
    main()
