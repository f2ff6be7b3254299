# A/B of forward kernel policies (0 = ping-pong, 2 = single-phase, 1 = generic).
mkdir -p gpurun_out
export TMPDIR=/tmp
for pol in ${POLICIES:-0 2}; do
  export MT_POLICY=$pol
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-extra --policy $pol > gpurun_out/ab_p$pol.json 2> gpurun_out/ab_p$pol.err || exit 1
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-extra --policy $pol --causal > gpurun_out/abc_p$pol.json 2>> gpurun_out/ab_p$pol.err || exit 1
done
for f in gpurun_out/ab*_p*.json; do python3 -c "import json,sys; j=json.load(open('$f')); print('$f', j['value'], j['roofline']['kernel_ms'])"; done
