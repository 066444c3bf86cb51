#!/bin/bash
# Experiment build of libnfdpf.so with -D flags applied to one source only (SRC, default
# filter_tiled: the pass and the step launches); the other objects are the in-tree build's:
# exp/lib_<TAG>.so (never shipped)
#   scripts/archive/exp_build_fast.sh S3B -DNFDPF_SWEEP_WE=3 -DNFDPF_SWEEP_PRIO=3
#   SRC=cglow scripts/archive/exp_build_fast.sh CGD -DNFDPF_EXP_CGDUMP -DNFDPF_CG_TARGET=68339
set -e
TAG=$1; shift
SRC=${SRC:-filter_tiled}
cd "$(dirname "$0")/../../normalizing-flows-dpfs_amd/csrc"
mkdir -p ../../exp /tmp/nfdpf_exp
FLAGS="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -w"
/opt/rocm/bin/hipcc $FLAGS "$@" -c $SRC.hip -o /tmp/nfdpf_exp/${SRC}_${TAG}.o
OBJS=$(for s in capi flows flows_bwd resample_soft resample_soft_bwd filter_step resample_ot measure measure_bwd misc cglow cglow_bwd rqs maf_bwd pseudo_lik nn_bwd filter_tiled; do [ $s = $SRC ] || echo build/$s.o; done)
/opt/rocm/bin/hipcc $FLAGS -shared -o ../../exp/lib_${TAG}.so $OBJS /tmp/nfdpf_exp/${SRC}_${TAG}.o
