# wgrad element check + timing of the 96-row Cout tiles against the 128-row ones (TONY_WGRAD_TBM96=0)
set -e
for cfg in "4 128 17 17 192 1 7 0 3" "4 160 17 17 160 7 1 3 0" "4 64 35 35 96 3 3 1 1" "4 448 8 8 384 3 3 1 1" "4 80 20 20 192 3 3 0 0"; do
  timeout -k 10 120 python tools/diag/wgrad_elem.py $cfg
  TONY_WGRAD_TBM96=0 timeout -k 10 120 python tools/diag/wgrad_elem.py $cfg | sed 's/^/TBM128 /'
done
