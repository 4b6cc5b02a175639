# K3 split sweep: main-kernel LDS budget x heavy threshold (multiple of the
# median window reads) on the 50 kb batch and the gap mix:
#   bash tools/k3_split_sweep.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k3split}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WL in fixed50 mix; do
  PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/mix_stats.py /tmp/b.npz 1024 $WL > $O/gen_$WL.log 2>&1 || exit 10
  for C in "def def" "45056 1.0" "45056 1.05" "45056 1.15" "47104 1.05"; do
    set -- $C
    E=""
    [ "$1" != def ] && E="PF_K3_LDS=$1 PF_K3_LDS_FB=73728 PF_K3_HEAVY_X=$2"
    env $E PF_DEBUG_FALLBACK=1 PF_PROF=0 timeout -k 10 200 python3 $R/tools/mix_stats.py /tmp/b.npz 1024 $WL > $O/${WL}_$1_$2.log 2>&1 || exit 11
    echo "$WL lds=$1 x=$2 $(grep -m1 '^kernels' $O/${WL}_$1_$2.log) $(grep -m2 deferred $O/${WL}_$1_$2.log | tail -1 | sed 's/.*K3 deferred/deferred/')"
  done
  rm -f /tmp/b.npz
done
