set -eu -o pipefail
O=gpurun_out/r05t; mkdir -p $O
for rep in a b; do
for ib in 63 48 32; do
  timeout -k 10 300 python3 bench.py --steps 1000 --warmup 50 --no-extra --no-cpu --item-blocks $ib > $O/ib${ib}_$rep.json 2> $O/ib${ib}_$rep.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['lean_kernel_ms'], d['roofline']['isolated_launch_ms'], d['p50_alone_ms'])" $O/ib${ib}_$rep.json ib$ib
done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu --item-blocks 48 > $O/ib48_20.json 2> $O/ib48_20.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ib48 20 steps', d['value'], d['ms_per_step'])" $O/ib48_20.json
