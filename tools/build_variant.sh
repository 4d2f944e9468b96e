#!/bin/bash
# Experiment build: libspimdecon.so with one source (SRC, default dog.hip) compiled under
# extra -D flags, the other objects reused from spim_registration_amd/_build.  Select it
# with SPIMDECON_LIB=<path>.
# usage: [SRC=fftconv.hip] tools/build_variant.sh TAG -DFOO=1 ...
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
mkdir -p exp
python -m spim_registration_amd.build > /dev/null
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Iinclude -I/opt/rocm/include"
SRC=${SRC:-dog.hip}
hipcc $F "$@" -x hip -c spim_registration_amd/csrc/$SRC -o exp/${SRC%.hip}_$TAG.o
OBJS=$(ls spim_registration_amd/_build/*.o | grep -v "/$SRC.o\$")
hipcc --offload-arch=gfx950 -shared -o exp/libspimdecon_$TAG.so $OBJS exp/${SRC%.hip}_$TAG.o -L/opt/rocm/lib -lrocfft -lrccl -Wl,-rpath,/opt/rocm/lib
echo exp/libspimdecon_$TAG.so
