#!/bin/sh
# Build libjmme.so and the oracle; fail loudly.  Usable from any cwd.
set -e
REPO="$(cd "$(dirname "$0")/.." && pwd)"
make -s -C "$REPO/--h.264-by-zhaodongyu_amd" -j"${MAX_JOBS:-8}"
make -s -C "$REPO/oracle" port
echo "built: $REPO/--h.264-by-zhaodongyu_amd/lib/libjmme.so"
