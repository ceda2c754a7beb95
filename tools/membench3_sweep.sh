#!/bin/bash
# membench3 sweep on the GPU box (synthetic KSEG model; see tools/membench3.hip)
B=${GRAFT_REPO_ROOT:-.}/build/membench3
for mode in 0 1; do
  for ilp in 1 4; do
    for len in 0 200 400 800 1600 3200; do
      timeout -k 5 60 $B $len $ilp 163840 $mode || exit $?
    done
  done
done
