#!/bin/bash
# Experiment build from an EDITED COPY of the kernel sources (the tree stays untouched, so the
# in-tree library is not rebuilt from the edit): csrc copied to a temp dir, the python
# expression EDIT applied to FILE there, SRC (default fftconv.hip) compiled, linked with the
# other in-tree objects into exp/libspimdecon_TAG.so.
# usage: FILE=fftconv_xt.inc EDIT='s.replace("a", "b")' tools/build_variant_src.sh TAG [-D...]
#    or: FILE=... EDITPY=edit.py tools/build_variant_src.sh TAG   (edit.py FILE edits in place)
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
mkdir -p exp
python -m spim_registration_amd.build > /dev/null
T=$(mktemp -d /tmp/sdvar.XXXXXX)
D=$T/pkg/csrc   # (the sources include ../../include/spimdecon.h)
mkdir -p $D $T/include
cp -r spim_registration_amd/csrc/. $D/
cp include/*.h $T/include/
if [ -n "$EDITPY" ]; then   # a python script editing the file named by its argument
  python3 "$EDITPY" "$D/$FILE"
else
python3 - "$D/$FILE" <<PY
import sys
p = sys.argv[1]
s = open(p).read()
t = eval('''$EDIT''')
assert t != s, "edit changed nothing"
open(p, "w").write(t)
PY
fi
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Iinclude -I/opt/rocm/include"
SRC=${SRC:-fftconv.hip}
hipcc $F "$@" -x hip -c $D/$SRC -o exp/${SRC%.hip}_$TAG.o
OBJS=$(ls spim_registration_amd/_build/*.o | grep -v "/$SRC.o\$")
hipcc --offload-arch=gfx950 -shared -o exp/libspimdecon_$TAG.so $OBJS exp/${SRC%.hip}_$TAG.o -L/opt/rocm/lib -lrocfft -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $T exp/${SRC%.hip}_$TAG.o
echo exp/libspimdecon_$TAG.so
