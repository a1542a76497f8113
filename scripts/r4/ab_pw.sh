export TMPDIR=/tmp
for i in 1 2; do
  for m in 0 1; do
    ZOO_PW=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_pw${m}_$i.log 2>&1 || exit 1
    echo "pw=$m run=$i $(grep -o '"value": [0-9.]*' gpurun_out/ab_pw${m}_$i.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/ab_pw${m}_$i.log)"
  done
done
