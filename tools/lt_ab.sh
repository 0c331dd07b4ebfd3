# Same-box A/B of learner-update timelines: for each variant, one rocprofv3 kernel trace of
# tools/learner_only.py and its per-dispatch table (layer_times.py). A variant is either
# environment assignments ("VAR=value ...") or learner_only.py arguments ("--set enc.x=0").
#   [LT_ARGS="--active 0.025"] bash tools/lt_ab.sh <tag> "--set enc.x=1" "--set enc.x=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  rm -rf /tmp/lt_$i
  ev=""; av=""
  case "$v" in --*) av="$v" ;; *) ev="$v" ;; esac
  (cd /tmp && env $ev timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/lt_$i -o run --output-format csv \
    -- python $R/tools/learner_only.py --steps 2 $LT_ARGS $av) > $R/gpurun_out/${tag}_lt$i.log 2>&1 || { tail -5 $R/gpurun_out/${tag}_lt$i.log; exit 1; }
  python $R/tools/layer_times.py /tmp/lt_$i --out $R/gpurun_out/${tag}_lt$i.md > /dev/null || exit 1
  echo "[$v] $(tail -1 $R/gpurun_out/${tag}_lt$i.md)"
done
