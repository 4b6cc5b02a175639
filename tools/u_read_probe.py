"""Where the -u pass's file read goes: the e2e_u genome
of bench.py (tests/_genome, scale argv[1]), then (1) a plain 16-thread pread
of the whole BAM from the page cache into an ordinary buffer, (2) the same
into a pinned buffer, (3) the driver (methphase_files -u) with
PF_INGEST_TRACE=1, which prints the ingest loop's read / copy / scan / send
split per contig fetch.  usage: python tools/u_read_probe.py [scale] [threads]"""
import concurrent.futures as cf
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import _genome  # noqa: E402


def pread_all(path, buf, threads, piece=4 << 20):
    fd = os.open(path, os.O_RDONLY)
    n = os.fstat(fd).st_size
    mv = memoryview(buf)[:n]

    def one(o):
        got = 0
        while got < min(piece, n - o):
            got += os.preadv(fd, [mv[o + got:min(o + piece, n)]], o + got)
    t = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(0, n, piece)))
    dt = time.perf_counter() - t
    os.close(fd)
    return n, dt


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    spec = _genome.GenomeSpec()
    spec.contigs = tuple((n, int(L * scale)) for n, L in spec.contigs)
    prefix = os.path.join("/tmp", f"pf_probe_{os.getpid()}")
    t = time.perf_counter()
    g = _genome.write_genome(prefix, spec, workers=threads)
    print(f"generated {g['bam_bytes'] / 1e9:.2f} GB in {time.perf_counter() - t:.1f}s", flush=True)
    n = g["bam_bytes"]
    buf = np.empty(n + 4096, np.uint8)
    buf[::4096] = 0
    for rep in range(2):
        nb, dt = pread_all(g["bam"], buf, threads)
        print(f"plain pread x{threads}: {nb / 1e9:.2f} GB in {dt * 1e3:.0f} ms = {nb / dt / 1e9:.1f} GB/s", flush=True)
    import torch
    pin = torch.empty(n + 4096, dtype=torch.uint8, pin_memory=True).numpy()
    for rep in range(2):
        nb, dt = pread_all(g["bam"], pin, threads)
        print(f"pinned pread x{threads}: {nb / 1e9:.2f} GB in {dt * 1e3:.0f} ms = {nb / dt / 1e9:.1f} GB/s", flush=True)
    del pin
    import subprocess
    cli = os.path.join(HERE, "pomfret_amd", "pomfret-amd")
    env = dict(os.environ, PF_INGEST_TRACE="1")
    for rep in range(2):
        t = time.perf_counter()
        p = subprocess.run([cli, "methphase", "-u", "-t", str(threads), "-o", prefix + ".cli", "--vcf", g["vcf"],
                            g["bam"]], capture_output=True, text=True, env=env)
        dt = time.perf_counter() - t
        print(f"cli rep {rep}: rc {p.returncode} {dt:.2f}s", flush=True)
        print("\n".join(ln for ln in p.stderr.splitlines() if "ingest" in ln or "[M::" in ln), flush=True)
        for e in (".cli.mp.vcf", ".cli.mp.gtf"):
            try:
                os.unlink(prefix + e)
            except OSError:
                pass
    from pomfret_amd import Context, LoadConfig
    from pomfret_amd.pipeline import methphase_files
    ctx = Context(0)
    os.environ["PF_INGEST_TRACE"] = "1"
    for rep in range(2):
        t = time.perf_counter()
        r = methphase_files(g["bam"], g["vcf"], prefix + ".drv", None, LoadConfig(), ctx=ctx, untagged=True,
                            threads=threads)
        dt = time.perf_counter() - t
        st = r["stats"]
        print(f"driver rep {rep}: {dt:.2f}s haptag {st.get('s_haptag')} windows {st.get('s_windows')} "
              f"finish {st.get('s_finish')} haptag phases {st.get('haptag')}", flush=True)
    ctx.close()
    for e in (".bam", ".bam.bai", ".vcf", ".drv.mp.vcf", ".drv.mp.gtf"):
        try:
            os.unlink(prefix + e)
        except OSError:
            pass
    for k in ("bam", "vcf"):
        for p in (g[k], g[k] + ".bai"):
            try:
                os.unlink(p)
            except OSError:
                pass


if __name__ == "__main__":
    main()
