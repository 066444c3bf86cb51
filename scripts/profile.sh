#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run -> gpurun_out/prof_<tag>/
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
  python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof_${TAG}.log; tail -3 gpurun_out/prof_${TAG}.log
find gpurun_out/prof_${TAG} -name '*stats*' | head
exit $rc
