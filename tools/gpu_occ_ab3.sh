# GPU box: SE align vote kernel at OCC 6 (default now) with wave caps 5 / 7, and OCC 7
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/sweep_host.py c3 4 wcap5:SVG_WAVE_CAP=5 wcap7:SVG_WAVE_CAP=7 base2: > gpurun_out/occ_c3_base.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_occ7.so timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 wcap7:SVG_WAVE_CAP=7 base2: > gpurun_out/occ_c3_occ7.txt 2>&1
