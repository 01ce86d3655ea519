# run_step NAME SECONDS CMD...: runs one GPU step under its own time limit, logs to gpurun_out/NAME.log;
# a crash/abort/timeout (anything but exit 0 or 1) ends the whole script.
run_step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] $name crashed/timed out; stopping"; exit $rc; fi
  return 0
}
