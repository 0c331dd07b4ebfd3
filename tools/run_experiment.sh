# Training run through the user-facing CLI on the GPU box, reduced to committable evidence.
#   bash tools/run_experiment.sh <name> <seconds> <microbeast.py args...>
# writes gpurun_out/<name>/{<name>Losses.csv, <name>_processed.csv, <name>_curve.md,
# <name>.csv.gz, stdout.log}; the checkpoint is deleted (too large to pull back).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
name=$1; shift
secs=$1; shift
out=$R/gpurun_out/$name
mkdir -p $out
timeout -k 10 $secs python -u $R/microbeast.py --exp_name $name --savedir $out \
  --total_steps 1000000000000 "$@" > $out/stdout.log 2>&1
rc=$?
rm -f $out/$name.ckpt $out/$name.ckpt.tmp
python $R/tools/learning_curve.py --name $out/$name --window 1000 --gzip > /dev/null
tail -2 $out/stdout.log
exit $rc
