#!/bin/bash
# Experiment builds of libnfdpf.so with -D flags (never shipped): exp/lib_<TAG>.so
#   scripts/archive/exp_build.sh TRACE -DNFDPF_EXP_TRACE
set -e
TAG=$1; shift
cd "$(dirname "$0")/../../normalizing-flows-dpfs_amd/csrc"
mkdir -p ../../exp
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -w "$@" -shared \
  capi.hip flows.hip flows_bwd.hip resample_soft.hip resample_soft_bwd.hip filter_step.hip filter_tiled.hip resample_ot.hip measure.hip measure_bwd.hip misc.hip \
  cglow.hip cglow_bwd.hip rqs.hip maf_bwd.hip pseudo_lik.hip nn_bwd.hip -o ../../exp/lib_${TAG}.so
