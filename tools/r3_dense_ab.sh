export TMPDIR=/tmp
for v in cur exp2 cur; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so; else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  echo "== $v"; PCD_LIB=$lib timeout -k 10 120 python tools/dense_probe.py 10000000 3 2>&1 | grep dense
done
