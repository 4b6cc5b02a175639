"""Per-wave SQ counter summary (instructions and wait fractions per kernel)
from rocprofv3 --pmc CSVs of the passes in tools/measure_r03.sh.
usage: python tools/sq_summary.py OUT.json WORKLOAD_TEXT P1.csv [P2.csv ...]"""
import collections
import csv
import json
import sys

out, wl, paths = sys.argv[1], sys.argv[2], sys.argv[3:]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for p in paths:
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
        if not k.startswith("pf_"):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
res = {}
for k, c in acc.items():
    waves = c.get("SQ_WAVES", 0.0)
    if not waves:
        continue
    cyc = c.get("SQ_WAVE_CYCLES", 0.0)
    d = {"per_wave": {"cycles_quad": round(cyc / waves), "valu": round(c.get("SQ_INSTS_VALU", 0) / waves),
                      "salu": round(c.get("SQ_INSTS_SALU", 0) / waves), "lds": round(c.get("SQ_INSTS_LDS", 0) / waves)}}
    if cyc:
        d["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / cyc, 3)
        d["wait_inst_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / cyc, 3)
        d["active_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / cyc, 3)
    for extra in ("SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT"):
        if extra in c:
            d["per_wave"][extra.lower()[3:]] = round(c[extra] / waves)
    res[k] = d
res["workload"] = wl
res["units"] = "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md)"
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
