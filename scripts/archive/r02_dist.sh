#!/bin/bash
# Gate-firing rehearsal (frame encodings = particle encoder(true positions), so the ESS gate
# fires): N=1 with the per-step gate and with the speculative gate, then N=2 ranks on ONE GPU
# over gloo (speculative and per-step exchange).  Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--enc-from-state --no-cpu-baseline --steps ${STEPS:-10} --warmup 3"
run() {  # tag, command...
  local tag=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/dist_$tag.json 2> gpurun_out/dist_$tag.err
  local rc=$?; echo "$tag rc=$rc"; tail -c 200 gpurun_out/dist_$tag.json; echo
  return $rc
}
run n1 python -u bench.py $A --speculate 0 &&
run n1_spec python -u bench.py $A --speculate 1 &&
NFDPF_DIST_BACKEND=gloo run n2_gloo_spec python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $A --speculate 1 &&
NFDPF_DIST_BACKEND=gloo run n2_gloo_step python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 $A --speculate 0
