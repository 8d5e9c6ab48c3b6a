#!/bin/bash
# Round 3: 16-bit chain kernel -- chain parity at 8/10/12/14 bits, the drop-in suites
# (8-bit and high bit depth), then the 10-bit 1080p drop-in bench.
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r3q
mkdir -p $o
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py \
  tests/test_hbd_gpu.py tests/test_jm_dropin_hbd_gpu.py tests/test_jm_dropin_gpu.py > $o/pytest.log 2>&1
timeout -k 10 300 python3 tools/bench_dropin.py --frames 3 --mode -1 --bits 10 > $o/dropin_10bit_fs.json 2> $o/a.err
timeout -k 10 300 python3 tools/bench_dropin.py --frames 3 --mode 0 --bits 10 > $o/dropin_10bit_ffs.json 2> $o/b.err
echo r3q done
