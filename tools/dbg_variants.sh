set -e
for v in new nodpp noasm noboth; do
  echo "== $v"
  JMME_LIB=--h.264-by-zhaodongyu_amd/lib/variants/$v/libjmme.so timeout -k 10 120 python3 tools/dbg_case.py c1_foreman_qcif_fs16 2>&1 | grep -v amdgpu.ids | tail -12
done
