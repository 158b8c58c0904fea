set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C1="1 192 28 28 16 1 1 1 1 0 0"
C2="5 480 14 14 64 1 1 1 1 0 0"
C4="1 832 7 7 48 1 1 1 1 0 0"
for a in "9 1" "13 1" "14 1" "15 1" "9 3" "13 3" "14 2"; do
  set -- $a
  echo "### cfg $1 splits $2"
  timeout -k 10 60 python tools/ktrace.py --conv "$C1" --conv "$C2" --conv "$C4" --cfg $1 --splits $2
done
