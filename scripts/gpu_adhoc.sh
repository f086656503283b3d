set -u
mkdir -p gpurun_out/profattn
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profattn -o run -- python3 tools/attn_bench.py > gpurun_out/profattn/out.txt 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/profattn/out.txt | grep -v amdgpu
python3 tools/kstats.py $(find gpurun_out/profattn -name "*kernel_stats.csv" | head -1) 1 12
