set -e
for cfg in "4 384 8 8 384 1 3 0 1" "2 384 8 8 384 1 3 0 1" "4 384 8 8 384 3 1 1 0" "4 448 8 8 384 3 3 1 1" "4 128 17 17 192 1 7 0 3"; do
  timeout -k 10 120 python tools/diag/wgrad_elem.py $cfg
  TONY_WGRAD_INC=0 timeout -k 10 120 python tools/diag/wgrad_elem.py $cfg | sed 's/^/INC=0 /'
  TONY_WGRAD_GLDS=0 timeout -k 10 120 python tools/diag/wgrad_elem.py $cfg | sed 's/^/GLDS=0 /'
done
