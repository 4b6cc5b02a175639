# K3 launch-parameter sweep on the gap-mix batch (main kernel LDS budget x
# number of heavy problems), run on the GPU box:  bash tools/k3_mix_sweep.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k3sweep}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/mix_stats.py /tmp/mix1024.npz 1024 mix > $O/gen.log 2>&1 || exit 10
for H in default 400 600; do
  for L in default 49152; do
    E=""
    [ "$H" != default ] && E="$E PF_K3_HEAVY=$H"
    [ "$L" != default ] && E="$E PF_K3_LDS=$L PF_K3_LDS_FB=73728"
    env $E PF_PROF=0 timeout -k 10 200 python3 $R/tools/mix_stats.py /tmp/mix1024.npz 1024 mix > $O/h${H}_l${L}.log 2>&1 || exit 11
    echo "heavy=$H lds=$L $(head -1 $O/h${H}_l${L}.log)"
  done
done
rm -f /tmp/mix1024.npz
