#!/bin/bash
# Build libjmme variants for A/B and counter attribution (CPU, before a GPU call):
#   tools/build_variants.sh name:FLAGS [name:FLAGS ...]
# e.g. base: noexp:-DJMME_ABL_NOEXPAND nofold:-DJMME_ABL_NOFOLD
# -> --h.264-by-zhaodongyu_amd/lib/variants/<name>/libjmme.so (JMME_LIB selects one)
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  make -s -C "$R/--h.264-by-zhaodongyu_amd" -j8 LIBDIR="$R/--h.264-by-zhaodongyu_amd/lib/variants/$name" EXTRA="$flags"
done
