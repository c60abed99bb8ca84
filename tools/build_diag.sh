#!/bin/bash
# Diagnostic copies of libnrse_hip.so with one part of the 256x256 GEMM ablated
# (NRSE_G3_ABLATE in csrc/gemm256.hip); load one with NRSE_LIB_PATH=build/diag/libnrse_diagN.so.
set -e
cd "$(dirname "$0")/../noise-robust-speech-embedding_amd"
make -C csrc -j8 >/dev/null
mkdir -p build/diag
OBJS=$(ls build/obj/*.o | grep -v gemm256)
for n in ${DIAG:-1 2 3 4 5 6}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -DNRSE_G3_ABLATE=$n \
    -c csrc/gemm256.hip -o build/diag/gemm256_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/diag/libnrse_diag$n.so $OBJS build/diag/gemm256_$n.o
done
echo built diag libs
# attention backward ablations (NRSE_ATT_ABLATE in csrc/attention_mfma.hip)
OBJS=$(ls build/obj/*.o | grep -v attention_mfma)
for n in ${ADIAG:-}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -DNRSE_ATT_ABLATE=$n \
    -c csrc/attention_mfma.hip -o build/diag/attn_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/diag/libnrse_adiag$n.so $OBJS build/diag/attn_$n.o
done
