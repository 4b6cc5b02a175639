"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json
(HBM bytes per launch of each kernel of the bench workload), the file bench.py
reads for roofline.traffic.

Counters are collected in separate passes (they do not fit one pass on gfx950)
with `--kernel-trace --pmc FETCH_SIZE` resp. `WRITE_SIZE` over
tools/run_aln_once.py (the bench's rank-0 record-level batch; tools/run_once.py
for the calls-level boundary), see tools/measure_r01.sh.  K0's count pass
(pf_k0_load<0>, run once at upload) is left out: the step runs pf_k0_load<1>.
Units are KiB.  Calibration on this box (tools/ubench/hbm_cal.hip, 1 GiB swept
past the 256 MiB Infinity Cache): FETCH_SIZE reports exactly 1/2 of the bytes
read for 1-, 4- and 16-byte-per-lane coalesced loads alike, WRITE_SIZE the
bytes written (u32 stores exact, u8 stores +2.5 %); so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv CAL_FETCH.csv CAL_WRITE.csv [records|calls]
"""
import collections
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def kernel_name(raw):
    """'void pf_k0_load<1>(pf_load_dev)' -> 'pf_k0_load'; None for the count pass."""
    n = raw.split("(")[0].strip()
    if n.startswith("void "):
        n = n[5:]
    if "<" in n:
        if n.endswith("<0>"):
            return None
        n = n.split("<")[0]
    return n


def per_kernel(path, counter):
    vals = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = kernel_name(r["Kernel_Name"])
        if name is None:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] += float(r["Counter_Value"])
        names[d] = name
    out = collections.defaultdict(list)
    for d, v in vals.items():
        out[names[d]].append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    fetch, write, cal_f, cal_w = sys.argv[1:5]
    boundary = sys.argv[5] if len(sys.argv) > 5 else "records"
    from bench import WORKLOAD
    # the bench's N=1 workload (strong scaling: every window on this GPU)
    WORKLOAD = dict(WORKLOAD, windows_per_gpu=WORKLOAD["n_windows"])
    f = per_kernel(fetch, "FETCH_SIZE")
    w = per_kernel(write, "WRITE_SIZE")
    cf = per_kernel(cal_f, "FETCH_SIZE")
    cw = per_kernel(cal_w, "WRITE_SIZE")
    gib_kib = float(1 << 20)
    cal = {k: {"fetch_kib": cf.get(k), "write_kib": cw.get(k), "bytes_touched_kib": gib_kib}
           for k in sorted(set(cf) | set(cw))}
    kernels = {}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("pf_"):
            continue
        fk, wk = f.get(k, 0.0), w.get(k, 0.0)
        kernels[k] = {"fetch_kib": round(fk, 1), "write_kib": round(wk, 1),
                      "hbm_bytes_per_launch": int((2.0 * fk + wk) * 1024)}
    res = {"workload": dict(WORKLOAD, boundary=boundary), "fetch_correction": 2.0,
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024",
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE, separate passes, "
                     + ("tools/run_aln_once.py" if boundary == "records" else "tools/run_once.py")
                     + " (bench rank-0 batch), averaged over launches",
           "calibration": cal, "kernels": kernels}
    out = os.path.join(HERE, "profiles", "pmc_traffic.json")
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
