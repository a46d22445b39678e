export PYTHONPATH=$PWD
for L in pyabc_amd/libabcgpu.so ab/libfr_cpt4.so ab/libfr_cpt16.so pyabc_amd/libabcgpu.so ab/libfr_cpt4.so ab/libfr_cpt16.so; do
  echo "== $L $(ABCGPU_LIB=$L timeout -k 10 120 python3 -u tools/bench_fused.py --wsigma 2.2 --rates 1e-4 --B 134217728 --reps 3 --modes plain 2>&1 | grep candidates)"
done
