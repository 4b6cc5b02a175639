# K3 dynamic-LDS sweep (main kernel size; fallback at 72 KB), 60x and 30x, 1024 windows
set -e
out=${1:-gpurun_out/k3sweep}
mkdir -p $out
for cov in 60 30; do
for l in 47104 40960 34816; do
  PF_K3_LDS=$l PF_K3_LDS_FB=73728 timeout -k 10 300 python bench.py --no-legs --no-cpu --steps 50 --coverage $cov \
      > $out/b_${cov}_${l}.json 2> $out/b_${cov}_${l}.err
  echo "$cov $l done"
done
done
