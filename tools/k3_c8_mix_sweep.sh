# K3 with u8 count pairs on the gap mix: main budget 44 KB x heavy threshold
#   bash tools/k3_c8_mix_sweep.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k3c8}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/mix_stats.py /tmp/b.npz 1024 mix > $O/gen.log 2>&1 || exit 10
for C in "def def" "45056 1.3" "45056 1.5" "45056 1.7" "56000 2.0"; do
  set -- $C
  E=""
  [ "$1" != def ] && E="PF_K3_LDS=$1 PF_K3_LDS_FB=73728 PF_K3_HEAVY_X=$2"
  env $E PF_DEBUG_FALLBACK=1 PF_PROF=0 timeout -k 10 200 python3 $R/tools/mix_stats.py /tmp/b.npz 1024 mix > $O/mix_$1_$2.log 2>&1 || exit 11
  echo "mix lds=$1 x=$2 $(grep -m1 '^kernels' $O/mix_$1_$2.log) $(grep -m2 deferred $O/mix_$1_$2.log | tail -1 | sed 's/.*K3 deferred/deferred/')"
done
rm -f /tmp/b.npz
