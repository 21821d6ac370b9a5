set -e
mkdir -p gpurun_out/r02v
for v in ph1 ph0; do
  PTYX_LIB=$PWD/ptyrad_amd/lib/var/libptyx_$v.so timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02v/$v.txt 2> gpurun_out/r02v/$v.err
  grep -a "F3" gpurun_out/r02v/$v.txt | head -8
done
