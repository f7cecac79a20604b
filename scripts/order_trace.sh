#!/bin/bash
# Kernel traces of the c4 bench for the A/B library (MERPCR_LIB=libmerpcr_hip_base.so, built
# beforehand from another revision) and the product library: the order stage per kernel.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in base new; do
  if [ $L = base ]; then export MERPCR_LIB=$R/merpcr_amd/_lib/libmerpcr_hip_base.so; else unset MERPCR_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ordtr_$L -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 10 --no-cpu-baseline --no-e2e --no-pmc > $R/gpurun_out/ordtr_$L.log 2>&1 || exit 1
done
