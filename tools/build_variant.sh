#!/bin/bash
# Build an engine library variant with extra kernel defines, for A/B runs
# (KWOK_ENGINE_LIB=...).  Usage: build_variant.sh NAME "-DFOO=1 -DBAR=2" [SOURCE [OBJ]]
# (SOURCE: compiled in place of OBJ's source; OBJ: kernels (default), ingest or json)
set -e
cd "$(dirname "$0")/../kwok_amd"
make -s lib/libkwok_engine.so
mkdir -p lib/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $2 \
  -c ${3:-csrc/kernels.hip} -o lib/var/${4:-kernels}_$1.o
OBJS="lib/kernels.o lib/ingest.o lib/json.o"
OBJS=${OBJS/lib\/${4:-kernels}.o/lib\/var\/${4:-kernels}_$1.o}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/var/libkwok_engine_$1.so lib/engine.o lib/templates.o \
  lib/codec.o lib/gotemplate.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
strip lib/var/libkwok_engine_$1.so; echo lib/var/libkwok_engine_$1.so
