set -o pipefail
for sz in "24 impala_deep" "16 impala_flat"; do set -- $sz
 for lib in new notsh; do la=""; [ $lib = notsh ] && la="--lib variants/notsh"
  timeout -k 10 300 python tools/learner_only.py --size $1 --arch $2 --active 0.023 --steps 5 $la > gpurun_out/tsh_${1}_$lib.log 2>&1 || { tail -20 gpurun_out/tsh_${1}_$lib.log; exit 4; }
  echo "$1 $2 $lib: $(tail -1 gpurun_out/tsh_${1}_$lib.log)"
 done
done
