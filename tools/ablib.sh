#!/bin/bash
# Build an A/B candidate library from the current sources with extra compile flags, reusing the
# in-tree objects (only the changed translation units recompile):
#   bash tools/ablib.sh NAME "EXTRA FLAGS"   ->  noise-robust-speech-embedding_amd/ablib/NAME.so
# (load it with NRSE_LIB_PATH=noise-robust-speech-embedding_amd/ablib/NAME.so; tools/gpu_ab.sh)
set -e
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/noise-robust-speech-embedding_amd
OBJ=$PKG/build/obj_$NAME
mkdir -p $PKG/ablib $OBJ
cp -p -n $PKG/build/obj/*.o $OBJ/ 2>/dev/null || true
# any object whose flags differ must rebuild: touch the sources named in FORCE (default all that
# the EXTRA flags could touch: every .hip)
if [ -n "$EXTRA" ] && [ ! -f $OBJ/.flags ] || [ "$(cat $OBJ/.flags 2>/dev/null)" != "$EXTRA" ]; then
  for f in ${FORCE:-$(cd $PKG/csrc && ls *.hip)}; do rm -f $OBJ/${f%.hip}.o; done
  echo "$EXTRA" > $OBJ/.flags
fi
make -C $PKG/csrc -j8 OUT=$PKG/ablib/$NAME.so OBJDIR=$OBJ EXTRA="$EXTRA" 2>&1 | grep -E "error|warning: (?!unused)" || true
ls -la $PKG/ablib/$NAME.so
