#!/bin/bash
# Builds tools/bin/wsr_check (gfx950 + the C oracle); run it on the GPU box.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin build/obj
gcc -O2 -c oracle/sydelta_oracle.c -o build/obj/oracle_wsr.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sy_amd/csrc -c tools/wsr_check.hip -o build/obj/wsr_check.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 build/obj/wsr_check.o build/obj/oracle_wsr.o -o tools/bin/wsr_check
