#!/bin/bash
# A/B library of the current source with one edit (never shipped):
#   tools/diag/variant.sh <name> <sed expression on sng_kernels.hip>  ->  lib/libsng_<name>.so
#   tools/diag/variant.sh <name> -p <patch against csrc/ (-p1)>         ->  lib/libsng_<name>.so
# e.g. tools/diag/variant.sh w4 's/wide_wpb(int) { return 1; }/wide_wpb(int) { return 4; }/'
#      tools/diag/variant.sh refold -p tools/diag/patches/ref_day2_one_wave.patch
# A patch under tools/diag/patches/ applies to the source of the commit that added it (later kernel changes
# can move its context); profiles/r05_ab_*.txt name the builds each A/B compared.
# STAMPS=1 builds the diagnostic stamps build (SNG_DIAG_STAMPS) of the variant instead, MEMFLOOR=1 its memory-floor
# build (SNG_DIAG_MEMFLOOR: trivial charger arithmetic).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; shift
tmp=$(mktemp -d /tmp/sng_variant_${name}_XXXX)
cp -r "$ROOT/smart-nanogrid-gym_amd/csrc" "$tmp/csrc"
if [ "$1" = "-p" ]; then
  patch -s -p1 -d "$tmp/csrc" < "$(realpath "$2")"
else
  sed -i "$1" "$tmp/csrc/sng_kernels.hip"
fi
if diff -rq "$tmp/csrc" "$ROOT/smart-nanogrid-gym_amd/csrc" > /dev/null; then
  echo "variant.sh: the edit changed nothing" >&2; rm -rf "$tmp"; exit 2
fi
if [ "${STAMPS:-0}" = 1 ] || [ "${MEMFLOOR:-0}" = 1 ]; then
  kind=$([ "${STAMPS:-0}" = 1 ] && echo stamps || echo memfloor)
  cp "$ROOT/tools/diag/sng_kernels_diag.hip" "$tmp/csrc/"
  mkdir -p "$tmp/lib"
  make -s -C "$ROOT/tools/diag" CSRC="$tmp/csrc" OUT="$tmp/lib" "$tmp/lib/libsng_${kind}.so"
  cp "$tmp/lib/libsng_${kind}.so" "$ROOT/smart-nanogrid-gym_amd/lib/libsng_${name}.so"
else
  make -s -C "$tmp/csrc" ROOT="$ROOT" OUT="$tmp/lib" "$tmp/lib/libsng.so"
  cp "$tmp/lib/libsng.so" "$ROOT/smart-nanogrid-gym_amd/lib/libsng_${name}.so"
fi
rm -rf "$tmp"
echo "built smart-nanogrid-gym_amd/lib/libsng_${name}.so"
