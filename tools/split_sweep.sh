# Contexts per GPU (bench.py --split) on the headline job, the batch
# generated once: one bench run per context count, CPU/legs off.
#   bash tools/split_sweep.sh <tag> "2 3 4"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-split}
mkdir -p $O
cd $R
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 tools/run_aln_once.py 1024 0 /tmp/split_aln.npz 60 > $O/gen.log 2>&1 || exit 10
export PF_BENCH_ALN_CACHE=/tmp/split_aln.npz
for S in ${2:-2 3 4}; do
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-legs --e2e-windows 0 --e2e-u-scale 0 --split $S --steps 10 --warmup 3 > $O/split$S.json 2> $O/split$S.err || { tail -5 $O/split$S.err; exit 11; }
  python3 -c "import json,sys; d=json.loads(open('$O/split$S.json').read().strip().splitlines()[-1]); print('split $S', d['value'], d['ms_per_step'])" | tee -a $O/summary.txt
done
rm -f /tmp/split_aln.npz
