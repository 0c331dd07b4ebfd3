# training trajectory (active cells per env over updates) of bench.py from random init:
#   bash tools/gpu_r6_traj.sh <tag> "<dir>|<args>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; shift
i=0
for spec in "$@"; do
  d=${spec%%|*}; args=${spec#*|}; i=$((i+1))
  (cd $R/$d && timeout -k 10 300 python bench.py --settle 0 --steps 400 --warmup 5 --report_every 40 $args) > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 5; }
  echo "== $d [$args]"; grep "\[window\]" gpurun_out/${tag}_$i.log | awk '{print $3, $4, $9}' | tr '\n' ' '; echo
done
