#!/bin/bash
# Build ablation variants of libds2hip.so (gemm.hip with DS2_X6_ABL=n; the other objects as
# built by the Makefile) into deepspeech.pytorch_amd/ablation/: 1 no MFMA, 2 no global loads,
# 3 no residual splits, 4 no workgroup barrier.  Timing only: their results are wrong.
# usage (build container): bash scripts/gemm_ablation.sh
set -e
cd "$(dirname "$0")/../deepspeech.pytorch_amd/csrc"
make -j8 >/dev/null
mkdir -p ../ablation ../../build/abl
for n in 1 2 3 4; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics \
    -DDS2_X6_ABL=$n -c gemm.hip -o ../../build/abl/gemm_abl$n.o &
done
wait
objs=$(ls ../../build/csrc/*.o | grep -v '/gemm.o$')
for n in 1 2 3 4; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../ablation/libds2hip_abl$n.so $objs ../../build/abl/gemm_abl$n.o -ldl
done
ls -la ../ablation
