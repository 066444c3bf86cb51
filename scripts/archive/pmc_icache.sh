#!/bin/bash
# PMC pass over the default C2 bench: instruction-cache traffic of the step kernels
# (each launch starts with cold caches) -> gpurun_out/pmc_${TAG}_icache/
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
  SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_${TAG}_icache -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --graph 0 > gpurun_out/pmc_${TAG}_icache.log 2>&1
rc=$?; echo "pmc icache rc=$rc"; exit $rc
