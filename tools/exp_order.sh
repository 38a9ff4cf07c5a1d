set -e
cd $GRAFT_REPO_ROOT
for L in lib_base lib lib_u1 lib_ot2k; do
  echo "== $L"
  SG_HIP_LIBRARY=siddhi-1_amd/$L/libsiddhi_gpu.so timeout -k 10 180 python tools/exp_variants.py 24 16 uniform
done
