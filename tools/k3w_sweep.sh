# one-wave greedy kernel: dynamic-LDS sweep at the bench workload (60x, 1024 windows)
set -e
out=${1:-gpurun_out/k3w}
mkdir -p $out
for l in ${LDS_LIST:-25600 30720 40960}; do
  PF_K3W_LDS=$l timeout -k 10 300 python bench.py --no-legs --no-cpu --steps 30 > $out/b_$l.json 2> $out/b_$l.err
  python - $out/b_$l.json $l <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["ms_per_step"], {k: v["ms"] for k, v in d["kernels"].items() if "k3" in k})
PY
done
