set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ktrace.py --conv "20 3 224 224 64 7 7 2 2 3 3" --cfg dc7s2x64d2 > gpurun_out/kt7.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/ktrace.py --conv "20 3 227 227 96 11 11 4 4 0 0" --cfg dc11s4x32d2 >> gpurun_out/kt7.log 2>&1 || exit 1
tools/pmc.sh gpurun_out/pmc7 python3 tools/profile_op.py conv 20,3,224,224,64,7,7,2,2,3,3 --cfg dc7s2x64d2 --iters 20
