# Run GPU steps in order, each under its own time limit; a plain test failure (exit 1) lets
# the next step run, anything else (fault, abort, timeout, segfault) ends the script there.
#   gpurun -- 'bash tools/gpu_steps.sh TAG "SECONDS CMD..." "SECONDS CMD..." ...'
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  secs=${step%% *}; cmd=${step#* }
  echo "[step $i] $cmd"
  timeout -k 10 $secs bash -c "$cmd" > $OUT/step$i.log 2>&1
  rc=$?
  tail -15 $OUT/step$i.log
  echo "[step $i] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_steps] stopping after rc=$rc"; exit $rc; fi
done
echo "[gpu_steps] done"
