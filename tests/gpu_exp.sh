mkdir -p gpurun_out/exp
for x in 0 1 2 4 7; do
  BCSIM_EXP=$x BCSIM_WGT=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 5 > gpurun_out/exp/w$x.log 2>&1
  echo "== exp $x"; grep "\[tile\]" gpurun_out/exp/w$x.log | head -3 | cut -c1-160
done
