#!/bin/bash
# A/B of experiment libraries on the C2 bench line: scripts/archive/exp_ab.sh base W8 W32 ...
# (base = the in-tree libnfdpf.so); one bench run per lib, ms_per_step printed
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in "$@"; do
  lib=normalizing-flows-dpfs_amd/libnfdpf.so; [ "$tag" != base ] && lib=exp/lib_$tag.so
  NFDPF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-forced ${BENCH_ARGS} \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['value'], d['roofline']['achieved'])" || tail -3 gpurun_out/ab_$tag.err
  [ $rc -eq 0 ] || exit $rc
done
