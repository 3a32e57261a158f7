# Experimental library build for tools/ab.py, reusing the product objects:
#   bash tools/build_variant.sh <name> "<EXTRA flags>" [DIAG=1] <source>...
# copies polarcode_and_ldpc_amd/_lib/obj{,_diag} to build/obj_<name>, recompiles
# the listed sources with EXTRA and links build/lib_<name>.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXTRA=$2; shift 2
DIAG=0
if [ "$1" = "DIAG=1" ]; then DIAG=1; shift; fi
SRC="$R/polarcode_and_ldpc_amd/_lib/obj"; [ $DIAG = 1 ] && SRC="$R/polarcode_and_ldpc_amd/_lib/obj_diag"
OBJ="$R/build/obj_$NAME"
rm -rf "$OBJ"; mkdir -p "$OBJ"; cp -p "$SRC"/*.o "$OBJ"/
for s in "$@"; do rm -f "$OBJ/$s.o" "$OBJ/$s.hip.o" "$OBJ/$s.cpp.o"; done
make -s -C "$R/polarcode_and_ldpc_amd/csrc" -j8 DIAG=$DIAG OUT="$R/build/lib_$NAME.so" OBJDIR="$OBJ" EXTRA="$EXTRA"
echo "built build/lib_$NAME.so"
