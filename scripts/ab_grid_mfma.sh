set -e
for c in c3 c5; do
  for g in ${GRIDS:-512 1024 1536 2048}; do
    MMRE_SWEEP_GRID=$g TAG=g$g timeout -k 10 200 python scripts/ab_sweep.py $c 10 2>&1 | grep sweep
  done
done
