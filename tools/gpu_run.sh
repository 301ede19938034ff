#!/bin/bash
# Run GPU steps in order; stop at the first step that faults, aborts, segfaults or times out.
# Test failures (rc 1) do not stop the chain.  Usage: tools/gpu_run.sh "<name>:<timeout>:<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  mkdir -p "gpurun_out/$(dirname "$name")"
  echo "== $name ($tmo s): $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "stopping after $name (rc=$rc)"; exit $rc ;;
  esac
done
