# GPU box: SE align vote-kernel occupancy 5 (default) vs 6 vs 8 at C3
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 base2: > gpurun_out/occ_c3_base.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_occ6.so timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 base2: wcap8:SVG_WAVE_CAP=8 > gpurun_out/occ_c3_occ6.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_occ8.so timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 base2: wcap8:SVG_WAVE_CAP=8 > gpurun_out/occ_c3_occ8.txt 2>&1
