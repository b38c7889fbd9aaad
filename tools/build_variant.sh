#!/bin/bash
# Build a compile-time variant of libdisq_gpu.so: tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> disq_amd/_build/libdisq_gpu_NAME.so (for tools/gpu_variant_ab.sh).
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../disq_amd/csrc"
out=../_build/v_$name
mkdir -p $out
objs=()
for f in *.hip; do
  extra=""; [ $f = dq_inflate3.hip ] && extra="-mllvm -amdgpu-sched-strategy=max-ilp"  # as the Makefile
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -munsafe-fp-atomics -I../../include $extra $flags -c -o $out/${f%.hip}.o $f &
  objs+=($out/${f%.hip}.o)
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../_build/libdisq_gpu_$name.so "${objs[@]}" -lpthread
echo built ../_build/libdisq_gpu_$name.so
