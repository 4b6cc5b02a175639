"""configs[3]-shaped -u run pieces for profiling (the bench's e2e_u leg, one
step at a time): `gen <prefix> [scale]` writes the genome BAM + VCF
(tests/_genome, outside any profiler); `cli <prefix> [threads]` runs the
pomfret-amd binary with -v (phase timings on stderr); `drv <prefix> [threads]`
runs the in-process driver twice (cold, then warm context) and prints the
phase stats of both as JSON."""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))


def main():
    mode, prefix = sys.argv[1], sys.argv[2]
    if mode == "gen":
        import _genome
        spec = _genome.GenomeSpec()
        scale = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
        spec.contigs = tuple((n, int(L * scale)) for n, L in spec.contigs)
        t = time.time()
        g = _genome.write_genome(prefix, spec, workers=16)
        print(json.dumps({"records": g["n_records"], "bam_bytes": g["bam_bytes"], "gen_s": round(time.time() - t, 1)}))
        return
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    if mode == "cli":
        cli = os.path.join(HERE, "pomfret_amd", "pomfret-amd")
        t = time.perf_counter()
        p = subprocess.run([cli, "methphase", "-u", "-v", "-t", str(threads), "-o", prefix + ".cli", "--vcf",
                            prefix + ".vcf", prefix + ".bam"], capture_output=True, text=True)
        print(json.dumps({"rc": p.returncode, "s": round(time.perf_counter() - t, 3),
                          "stderr": [ln for ln in p.stderr.splitlines() if "phases" in ln or "E::" in ln]}))
        return
    from pomfret_amd import Context
    from pomfret_amd.pipeline import methphase_files
    t0 = time.perf_counter()
    ctx = Context(0)
    t1 = time.perf_counter()
    out = {"ctx_s": round(t1 - t0, 3)}
    for rep in ("cold", "warm"):
        t = time.perf_counter()
        r = methphase_files(prefix + ".bam", prefix + ".vcf", prefix + ".drv", None, ctx=ctx, untagged=True,
                            threads=threads)
        out[rep] = {"s": round(time.perf_counter() - t, 3), "stats": r["stats"]}
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
