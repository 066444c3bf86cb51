#!/bin/bash
# Round 3 multi-rank rehearsal on ONE GPU over gloo (RCCL refuses two ranks on one device): the
# driver's scaling command shape for C2 (default auto mode: speculative gate) and C4 (two-phase
# sharded Sinkhorn), plus C2 with informative encodings (gates fire: the miss / back-off path).
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag, command...
  local tag=$1; shift
  timeout -k 10 400 "$@" > gpurun_out/dist3_$tag.json 2> gpurun_out/dist3_$tag.err
  local rc=$?; echo "$tag rc=$rc"; tail -c 300 gpurun_out/dist3_$tag.json; echo
  return $rc
}
NFDPF_DIST_BACKEND=gloo run c2_n2 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline &&
NFDPF_DIST_BACKEND=gloo run c4_n2 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 2 --config c4 --steps 2 --warmup 1 --no-cpu-baseline &&
NFDPF_DIST_BACKEND=gloo run c2_n2_fire python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --enc-from-state --steps 5 --warmup 2 --no-cpu-baseline
