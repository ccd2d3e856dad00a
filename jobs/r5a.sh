set -o pipefail
mkdir -p gpurun_out/r5a
hipcc --offload-arch=gfx950 -O2 -std=c++17 benchmarks/capture_probe.hip -o gpurun_out/r5a/capture_probe -lpthread 2>/dev/null
timeout -k 10 60 gpurun_out/r5a/capture_probe > gpurun_out/r5a/capture_probe.txt 2>&1
echo probe rc=$?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a/b20.json 2> gpurun_out/r5a/b20.err && \
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/r5a/b200.json 2> gpurun_out/r5a/b200.err
echo bench rc=$?
