# Development probe: SDMA copy rates for several copy sizes / stream layouts
# (tools/kbench/pcie.hip) and CU-driven zero-copy rates (zerocopy.hip).
set -u
mkdir -p gpurun_out
for c in 32 4; do
  timeout -k 10 120 tools/kbench/pcie 256 $c >> gpurun_out/pcie.log 2>&1 || exit 1
done
timeout -k 10 200 tools/kbench/zerocopy 512 > gpurun_out/zerocopy.log 2>&1
