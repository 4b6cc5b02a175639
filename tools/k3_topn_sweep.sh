# K3: the n heaviest problems on the second stream, main kernel at 44 KB
#   bash tools/k3_topn_sweep.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k3topn}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/mix_stats.py /tmp/b.npz 1024 fixed50 > $O/gen.log 2>&1 || exit 10
for N in 0 40 80 160; do
  PF_K3_LDS=45056 PF_K3_LDS_FB=73728 PF_K3_HEAVY=$N PF_DEBUG_FALLBACK=1 PF_PROF=0 timeout -k 10 200 python3 $R/tools/mix_stats.py /tmp/b.npz 1024 fixed50 > $O/n_$N.log 2>&1 || exit 11
  echo "fixed50 lds=45056 heavy=$N $(grep -m1 '^kernels' $O/n_$N.log) $(grep -m2 deferred $O/n_$N.log | tail -1 | sed 's/.*K3 deferred/deferred/')"
done
rm -f /tmp/b.npz
