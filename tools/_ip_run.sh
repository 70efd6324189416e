set -e
cd /root/repo
mkdir -p gpurun_out/ip2; rm -f gpurun_out/ip2/*
timeout -k 10 400 python bench.py --steps 20 --warmup 10 --no-cpu > gpurun_out/ip2/bench.json 2> gpurun_out/ip2/bench.err
