set -u
export REPS=2
for a in "r2 4096" "r1 1000" "r1 5000" "r1 25000" "r3 20000" "pf 25000" "r2 1000000"; do
  timeout -k 5 60 python -u scripts/diag_decode.py $a || exit $?
done
