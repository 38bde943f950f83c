#!/bin/bash
# Start N va_alias_probe processes on GPU 0, S seconds each, all at once: va_alias_probe.sh N S MODE
# (MODE steady|churn, see va_alias_probe.cpp). One JSON line per process; exit 0 = no process ever
# read a word it did not write, 5 = some did.
N=${1:-9}; S=${2:-40}; M=${3:-steady}
cd "$(dirname "$0")"
pids=()
for ((r = 0; r < N; r++)); do
  timeout -k 10 $((S + 60)) ./va_alias_probe "$r" "$S" "$M" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "va_alias_probe N=$N S=$S mode=$M: rc=$rc"
exit $rc
