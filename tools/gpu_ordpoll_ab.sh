set -e
for v in 0 8; do
  LOCUST_ORD_VARIANT=$v LOCUST_ORD_TRACE=1 LOCUST_GRAPH=0 timeout -k 10 60 ./build/MapReduce data/hamlet.txt --warmup 5 --iters 1 --quiet > /dev/null 2> gpurun_out/ordv$v.txt
  echo "v=$v $(grep 'ord span' gpurun_out/ordv$v.txt | tail -1)"
  LOCUST_ORD_VARIANT=$v timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-extra > gpurun_out/hv$v.json
  echo "v=$v bench $(python3 -c "import json;print(json.load(open('gpurun_out/hv$v.json'))['value'])")"
done
