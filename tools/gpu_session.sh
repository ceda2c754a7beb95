#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time
# limit.  Ordinary test failures (exit 1) do not stop the session, but a crash,
# abort, fault or time-out (124/134/137/139 or signal) ends it immediately.
# usage: tools/gpu_session.sh <seconds> <logname> <command...> [---- <seconds> <logname> <command...>]...
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  secs=$1; log=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "----" ]; do cmd+=("$1"); shift; done
  [ "$1" == "----" ] && shift
  echo "=== [$log] ${cmd[*]}" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$log.log" 2>&1
  rc=$?
  echo "=== [$log] exit $rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$log.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "stopping session after exit $rc"; exit $rc ;;
  esac
done
