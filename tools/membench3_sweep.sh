#!/bin/bash
# membench3 sweep on the GPU box (synthetic KSEG model; see tools/membench3.hip)
# usage: tools/membench3_sweep.sh [waves-per-SIMD list] [len list] [ilp list]
B=${GRAFT_REPO_ROOT:-.}/build/membench3
for wps in ${1:-2}; do
  for mode in 0 1; do
    for ilp in ${3:-1 4}; do
      for len in ${2:-0 200 400 800 1600 3200}; do
        timeout -k 5 60 $B $len $ilp 163840 $mode $wps || exit $?
      done
    done
  done
done
