export TMPDIR=/tmp
for v in BASE NOMEAS NOCOND NODYNF; do
  if [ $v = BASE ]; then unset NFDPF_LIB; else export NFDPF_LIB=$PWD/exp/lib_$v.so; fi
  timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/exp_$v.log 2>&1 || exit $?
done
