set -o pipefail
D=gpurun_out/lmprof
mkdir -p $D
g++ -O3 -std=c++17 -ffp-contract=off -Iform_amd/csrc tools/cholbench/host_chol.cpp form_amd/csrc/smoother.cpp -o $D/host_chol && $D/host_chol > $D/host_chol.txt 2>&1
grep -m1 "model name" /proc/cpuinfo >> $D/host_chol.txt
cat $D/host_chol.txt
FMX_LIB=form_amd/ab/libfmx_lmprof.so timeout -k 10 300 python tools/stream_profile.py --config c2 --scans 360 > $D/sp_c2.txt 2>&1
grep -E "^lm|scans" $D/sp_c2.txt
