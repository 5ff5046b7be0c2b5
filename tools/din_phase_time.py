"""Average din_forward_kernel<32> launch time at the bench's DIN configs[2] workload, for
whichever librankops.so RANKOPS_LIB points at — used with the RK_DIN_SKIP_A / RK_DIN_SKIP_B
timing builds (make EXTRA=-DRK_DIN_SKIP_B ...) to split the kernel into its two phases."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

model, inp, fn, cfg, name = bench.workload("din", 4096, 0)
launch = model.fused_kernel_launcher(inp["dense"], inp["category"], inp["sequence"], inp["target"])
# hipGraph replays of 20 launches: the per-call host marshalling of the launcher (~40 us) would
# otherwise set the pace
print(f"{os.path.basename(os.environ.get('RANKOPS_LIB', 'librankops.so'))}: "
      f"{1e3 * bench.graph_kernel_avg_ms(launch):.2f} us per launch (graph replay)")
