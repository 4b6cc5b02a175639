# K0 instructions by phase on the bench's mix batch (256 windows, 60x): one SQ
# counter pass per PF_K0_DIAG cut (4 / 2 / 5 / 3 / 0: stop after the filters /
# the MM phase / the SEQ count / the SEQ pass / the whole kernel), the batch
# generated before any profiler starts.
#   bash tools/k0_sq_probe.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k0sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 200 python3 $R/tools/run_aln_once.py 256 0 /tmp/a256.npz 60 > $O/gen.log 2>&1 || exit 10
for M in 4 2 5 3 0; do
  PF_K0_DIAG=$M timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/s$M -o s$M --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/a256.npz 60 > $O/s$M.log 2>&1 || exit 11
  echo "diag $M done"
done
rm -f /tmp/a256.npz
python3 - $O <<'PY' | tee $O/summary.txt
import csv, sys, collections
O = sys.argv[1]
names = {"4": "filters", "2": "+MM/ML", "5": "+SEQ count", "3": "+SEQ placement", "0": "whole kernel"}
prev = None
for M in "42530":
    v = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f"{O}/s{M}/s{M}_counter_collection.csv")):
        if r["Kernel_Name"].startswith("pf_k0_load"):
            v[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    d = list(v.values())[-1]
    w = d["SQ_WAVES"]
    per = {k[3:].lower(): d[k] / w for k in d if k != "SQ_WAVES"}
    line = " ".join(f"{k} {per[k]:.0f}" for k in sorted(per))
    delta = "" if prev is None else "  | phase: " + " ".join(f"{k} {per[k] - prev[k]:+.0f}" for k in sorted(per))
    print(f"PF_K0_DIAG={M} ({names[M]}): per wave {line}{delta}")
    prev = per
PY
