"""Chromosome-scale `methphase -u` (VERDICT r04 "next round" 2): one 60x
contig large enough that the -u pre-pass fetches it in several ~4 GiB pieces
of compressed BAM (no environment override), against a genome of the same
shape whose contigs fit one piece each (bench.py's e2e_u genome, 96 Mb).
Per genome: the CLI wall time as a user runs it (`pomfret-amd methphase -u`,
no -c), the in-process driver with its pf_mp_stats (pieces, kept-arena hits
and misses, re-read bytes), and -- unless --no-cpu -- the CPU port with
outputs compared byte for byte.  Ends with an HG002 60x wall-clock
PROJECTION from the measured per-Mb rates (a projection, not a measurement).

usage: python tools/chrom_scale.py [contig_Mb=100] [--no-cpu] > profiles/r05/chrom_scale.json"""
import json
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
from pomfret_amd.bam import BamFile  # noqa: E402
from pomfret_amd.pipeline import methphase_files  # noqa: E402

HG002_MB = 3_100          # GRCh38 primary assembly, Mb (the projection's genome size)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def run_genome(tag, contigs, workdir, threads, cpu_threads, ctx, cpu):
    spec = _genome.GenomeSpec()
    spec.contigs = contigs
    prefix = os.path.join(workdir, f"pf_cs_{tag}_{os.getpid()}")
    t = time.perf_counter()
    g = _genome.write_genome(prefix, spec, workers=threads)
    res = {"contigs": [[n, L] for n, L in contigs], "genome_mb": sum(L for _, L in contigs) / 1e6,
           "records": g["n_records"], "bam_bytes": g["bam_bytes"], "gen_s": round(time.perf_counter() - t, 1)}
    log(f"[cs] {tag}: generated {res['records']} records, {res['bam_bytes'] / 2**30:.2f} GiB in {res['gen_s']}s")
    with BamFile(g["bam"]) as b:
        from pomfret_amd._lib import lib
        import ctypes as C
        L = lib()
        L.pf_bam_contig_pieces.argtypes = [C.c_void_p, C.c_int32, C.c_uint64, C.POINTER(C.c_int64)]
        L.pf_bam_contig_pieces.restype = C.c_uint64
        step = C.c_int64()
        res["pieces"] = {n: int(L.pf_bam_contig_pieces(b.handle, b.tid(n), 0, C.byref(step))) for n, _ in contigs}
    outs = {}

    def take(pre):
        o = [open(pre + e, "rb").read() for e in (".mp.vcf", ".mp.gtf")]
        for e in (".mp.vcf", ".mp.gtf"):
            os.unlink(pre + e)
        return o
    try:
        cli = os.path.join(HERE, "pomfret_amd", "pomfret-amd")
        cmd = [cli, "methphase", "-u", "-v", "-t", str(threads), "-o", prefix + ".cli", "--vcf", g["vcf"], g["bam"]]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, capture_output=True, text=True)
        dt = time.perf_counter() - t0
        if p.returncode != 0:
            raise RuntimeError(f"pomfret-amd failed ({p.returncode}): {p.stderr[-2000:]}")
        outs["cli"] = take(prefix + ".cli")
        res["cli"] = {"s": round(dt, 2), "s_per_mb": round(dt / res["genome_mb"], 5),
                      "phases": [ln for ln in p.stderr.splitlines() if "phases:" in ln]}
        log(f"[cs] {tag}: cli {dt:.2f}s")
        t0 = time.perf_counter()
        r = methphase_files(g["bam"], g["vcf"], prefix + ".drv", None, LoadConfig(), ctx=ctx, untagged=True,
                            threads=threads)
        dd = time.perf_counter() - t0
        outs["driver"] = take(prefix + ".drv")
        st = r["stats"]
        res["driver"] = {"s": round(dd, 2), "s_per_mb": round(dd / res["genome_mb"], 5),
                         "windows": int(r["decision"].shape[0]), "joined": int((r["decision"] >= 0).sum()),
                         "arena_hits": st["arena_hits"], "arena_misses": st["arena_misses"],
                         "reread_bytes": st["reread_bytes"], "window_fetches": st["windows"]["n_fetch"],
                         "haptag_comp_over_bam": round(st["haptag"]["comp_bytes"] / res["bam_bytes"], 3),
                         "phases": st}
        log(f"[cs] {tag}: driver {dd:.2f}s, hits {st['arena_hits']} misses {st['arena_misses']}")
        if cpu:
            from _oracle_pipeline import methphase_files_port
            rp, ph = methphase_files_port(g["bam"], g["vcf"], prefix + ".port", None, LoadConfig(), untagged=True,
                                          threads=cpu_threads)
            outs["cpu_port"] = take(prefix + ".port")
            res["cpu_port"] = {"s": round(ph["total_s"], 2), "threads": cpu_threads,
                               "phases_s": {k: round(v, 2) for k, v in ph.items()}}
            log(f"[cs] {tag}: cpu port {ph['total_s']:.1f}s")
        res["outputs_identical"] = all(o == outs["cli"] for o in outs.values())
        res["compared"] = sorted(outs)
    finally:
        for f in (g["bam"], g["bam"] + ".bai", g["vcf"]):
            if os.path.exists(f):
                os.unlink(f)
    return res


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 100.0
    cpu = "--no-cpu" not in sys.argv
    eff, _ = effective_cores()
    threads = min(16, eff)
    workdir = os.environ.get("TMPDIR", "/tmp")
    ctx = Context(0)
    out = {"what": "methphase -u, no -c, 60x, from files; pieces = the -u pre-pass's position pieces per contig "
                   "(~4 GiB compressed each, no override)", "threads": threads, "cpu_threads": min(32, eff)}
    out["chromosome"] = run_genome("chrom", (("chr1", int(mb * 1e6)),), workdir, threads, min(32, eff), ctx, cpu)
    out["single_piece"] = run_genome("genome", _genome.GenomeSpec().contigs, workdir, threads, min(32, eff), ctx,
                                     cpu)
    a, b = out["chromosome"]["cli"]["s_per_mb"], out["single_piece"]["cli"]["s_per_mb"]
    out["multi_over_single_per_mb"] = round(a / b, 3)
    out["hg002_60x_projection"] = {
        "kind": "PROJECTION from the per-Mb CLI rates above, not a measurement",
        "genome_mb": HG002_MB,
        "one_gpu_s_from_chromosome_rate": round(a * HG002_MB, 1),
        "one_gpu_s_from_single_piece_rate": round(b * HG002_MB, 1),
        "assumes": "HG002-like density (60x, 1 het SNV per kb, phase gaps every 50-100 kb as the synthetic "
                   "genome); contigs beyond the HBM reserve re-read their pieces (not modelled); the CPU port's "
                   "rate for the same genome: " + (f"{out['chromosome']['cpu_port']['s'] / out['chromosome']['genome_mb'] * HG002_MB:.0f} s"
                                                      if cpu else "not run")}
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
