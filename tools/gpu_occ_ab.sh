# GPU box: vote-kernel occupancy variants (SE align OCC 4 vs 5 at C3; PE subjunc OCC 2 vs 4 at C5pe)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 base2: > gpurun_out/occ_c3_base.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_occ4.so timeout -k 10 400 python3 -u tools/sweep_host.py c3 4 base2: > gpurun_out/occ_c3_occ4.txt 2>&1 && \
timeout -k 10 500 python3 -u tools/sweep_host.py c5pe 2 > gpurun_out/occ_c5pe_base.txt 2>&1 && \
SVG_LIB=subread_amd/lib/libsubread_amd_pesj2.so timeout -k 10 500 python3 -u tools/sweep_host.py c5pe 2 > gpurun_out/occ_c5pe_pesj2.txt 2>&1
