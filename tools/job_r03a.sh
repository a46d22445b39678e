timeout -k 10 400 python -u tools/probes/custom_model_c2.py 20 > gpurun_out/custom20.log 2>&1 || exit 1
grep model gpurun_out/custom20.log | cut -c1-600
bash tools/ab_local_fit.sh ab/libdm_sb4.so ab/libdm_u4.so ab/libdm_u8.so ab/libdm_w8.so
