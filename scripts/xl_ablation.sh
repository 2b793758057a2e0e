#!/bin/bash
# Build timing ablations of the XCD-local GRU kernels (gru_xl.hip with DS2_XL_ABL=n; the other
# objects as the Makefile builds them) into deepspeech.pytorch_amd/ablation/libds2hip_xl<n>.so:
# 1 no per-step input loads, 2 no per-step output stores, 3 both, 4 no hand-off waits, 7 all.
# Timing only: their results are wrong.  usage (build container): bash scripts/xl_ablation.sh
set -e
cd "$(dirname "$0")/../deepspeech.pytorch_amd/csrc"
make -j8 >/dev/null
mkdir -p ../ablation ../../build/abl
for n in 1 2 3 4 7 8; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics \
    -DDS2_XL_ABL=$n -c gru_xl.hip -o ../../build/abl/gru_xl_abl$n.o &
done
wait
objs=$(ls ../../build/csrc/*.o | grep -v '/gru_xl.o$')
for n in 1 2 3 4 7 8; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../ablation/libds2hip_xl$n.so $objs ../../build/abl/gru_xl_abl$n.o -ldl
done
ls -la ../ablation
