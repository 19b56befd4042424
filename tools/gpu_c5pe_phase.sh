# GPU box: wave-kernel phase split for C5pe (stamps build)
mkdir -p gpurun_out
SVG_LIB=subread_amd/lib/libsubread_amd_stamps.so timeout -k 10 300 python -u tools/phase_profile.py c3 2000000 sjpe > gpurun_out/phase_c5pe2.txt 2>&1
