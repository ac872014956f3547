set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tb_pytest.log 2>&1 || { tail -20 gpurun_out/tb_pytest.log; exit 1; }
tail -2 gpurun_out/tb_pytest.log
for f in akarirender-1_amd/libakr_hip.so akarirender-1_amd/variants/libakr_hip_tb128.so akarirender-1_amd/variants/libakr_hip_tb64.so; do
  echo "== $f"
  AKR_HIP_LIB=$PWD/$f timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/tb_$(basename $f).json 2>gpurun_out/tb_$(basename $f).err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(d['value'], {n: round(v['avg_ms'],3) for n,v in k.items()})" gpurun_out/tb_$(basename $f).json
done
