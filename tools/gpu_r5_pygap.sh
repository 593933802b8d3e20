# round 5: the Python side of the gap between two C2 evaluations (host-probe variant)
set -o pipefail
export SGP_AB_LIB=tools/ab/hprobe/libsgp.so
timeout -k 10 200 python3 tools/c2_pygap.py 400
