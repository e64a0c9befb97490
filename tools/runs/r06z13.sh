# configs[3]'s B=8 T=500 stage2 vocoder: the head window and mid window picks
# of the grid model against the alternatives, in one process each.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06z13_s2_windows.txt
timeout -k 10 150 python3 -u tools/probe/voc_env_ab.py M2_S2_HEAD_TF unset,16,19,24,27 2 s2 8 500 8 40 > $O 2>&1 || exit 1
timeout -k 10 150 python3 -u tools/probe/voc_env_ab.py M2_S2_MID_ALT unset,0,1 2 s2 8 500 8 40 >> $O 2>&1 || exit 1
cat $O
