# Sourced by the gpurun scripts: step <name> <seconds> <command...> runs one
# GPU step under its own time limit, logs to gpurun_out/<name>.log, and ends
# the script at the first failure (no further GPU step after a fault/timeout).
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
