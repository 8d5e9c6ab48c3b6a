set -e
mkdir -p gpurun_out/r6e
bash tools/ab.sh base wp84 > gpurun_out/r6e/ab.txt 2>&1
for v in stamps wp84s; do JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 120 python3 tools/stamps.py > gpurun_out/r6e/stamps_$v.txt 2>&1; done
for v in base wp84; do JMME_LIB=$PWD/--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so bash tools/pmc.sh gpurun_out/r6e/pmc_$v sq2 > /dev/null 2>&1; python3 tools/pmc_summary.py gpurun_out/r6e/pmc_$v > gpurun_out/r6e/pmc_$v.txt 2>&1; done
echo done
