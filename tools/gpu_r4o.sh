# FC weight-gradient dispatch order A/B (MBK_WGRAD_ORDER=part: row ranges fastest, the default
# for the plain FC; chunk: the 8 output chunks of a row range together, sharing its rows in L2).
#   bash tools/gpu_r4o.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4o}
bash tools/lt_ab.sh ${tag} "MBK_WGRAD_ORDER=part" "MBK_WGRAD_ORDER=chunk" || exit 4
grep -E "fc_wgrad|colsum|gemm_nt|update span" gpurun_out/${tag}_lt1.md gpurun_out/${tag}_lt2.md
