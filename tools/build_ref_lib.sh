#!/bin/bash
# Build libnrse_hip.so from a git revision (default HEAD) into the package dir as
# diag_libs_<name>.so, for same-box A/B runs (NRSE_LIB_PATH=...). Usage: tools/build_ref_lib.sh [rev] [name]
set -e
REV=${1:-HEAD}
NAME=${2:-head}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/nrse_ref.XXXX)
git -C "$ROOT" archive "$REV" include noise-robust-speech-embedding_amd/csrc | tar -x -C "$TMP"
make -C "$TMP/noise-robust-speech-embedding_amd/csrc" -j8 OUT="$ROOT/noise-robust-speech-embedding_amd/diag_libs_$NAME.so" \
     OBJDIR="$TMP/obj" > /dev/null
rm -rf "$TMP"
ls -la "$ROOT/noise-robust-speech-embedding_amd/diag_libs_$NAME.so"
