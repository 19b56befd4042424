#!/bin/bash
# GPU box, round 4 call P: host sub-batch size and wave-kernel residency cap re-swept on the
# round-end build (C3, interleaved configurations in one process)
mkdir -p gpurun_out/r4p
timeout -k 10 600 python -u tools/sweep_host.py c3 10 'sub768k:host_sub=786432' 'sub1280k:host_sub=1310720' 'sub1536k:host_sub=1572864' 'cap5:wave_cap=5' 'cap7:wave_cap=7' 'cap8:wave_cap=8' 'base2:' > gpurun_out/r4p/sweep.txt 2>&1
