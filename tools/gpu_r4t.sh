#!/bin/bash
# GPU box, round 4 call T: the probe line kernel's grid (blocks per CU) swept at C3
mkdir -p gpurun_out/r4t
timeout -k 10 600 python -u tools/sweep_host.py c3 10 'pc8:probe_cap=8' 'pc16:probe_cap=16' 'pc24:probe_cap=24' 'pc32:probe_cap=32' 'pc12:probe_cap=12' > gpurun_out/r4t/sweep_probe_cap.txt 2>&1
