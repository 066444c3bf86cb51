#!/bin/bash
# Round 5: the one-launch pass over more rows than one MI355X holds at once (resident chunks of
# rows, pass_launch_rows) against the step launches (NFDPF_PASS=0), bench lines per B
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-forced --no-informative "$@" \
    > gpurun_out/rows_$tag.json 2> gpurun_out/rows_$tag.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/rows_$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'batch', d['config'].get('global_batch'))"
}
run c2_b64 --batch 64
run c2_b128 --batch 128
run c2_b256 --batch 256
run c2_b128_force --batch 128 --force-resample
run c3_b128 --config c3 --batch 128
NFDPF_PASS=0 run c2_b128_steps --batch 128
NFDPF_PASS=0 run c3_b128_steps --config c3 --batch 128
