#!/bin/bash
# Board power / clock while integrate_kernel runs back to back (LJ13 B=1024 Euler-100, ~10 s), sampled by rocm-smi.
# Usage (from gpurun): bash tools/power_probe.sh [divergence: none|hutchinson]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
DIV=${1:-none}
timeout -k 5 20 rocm-smi --showpower --showclocks > gpurun_out/power_idle.txt 2>&1
cat > /tmp/power_load.py <<'EOF'
import os, sys, time, torch
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "ecnf-baseline-neurips-2023_amd"))
from ecnf_amd import CONFIGS, init_params, _lib
from ecnf_amd.engine import EcnfHandle, SolveOptions
cfg = CONFIGS["lj13"]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
x0 = h.base_sample(torch.randn((1024, cfg.event_dim), device="cuda"))
feat = torch.zeros((1024, cfg.n_nodes), device="cuda", dtype=torch.int32)
div = _lib.DIV_HUTCHINSON if sys.argv[1] == "hutchinson" else _lib.DIV_NONE
eps = torch.randn_like(x0) if div else None
t0 = time.time(); n = 0
while time.time() - t0 < 10:
    for _ in range(10):
        h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.01), div, eps, check_status=False)
    torch.cuda.synchronize(); n += 10
print(f"launches {n} in {time.time() - t0:.1f} s: {1e3 * (time.time() - t0) / n:.2f} ms each")
EOF
timeout -k 5 60 python /tmp/power_load.py $DIV > gpurun_out/power_load_$DIV.txt 2>&1 &
LP=$!
sleep 6
for i in 1 2 3 4; do timeout -k 5 10 rocm-smi --showpower --showclocks >> gpurun_out/power_busy_$DIV.txt 2>&1; sleep 0.5; done
wait $LP
cat gpurun_out/power_load_$DIV.txt
grep -iE "power|sclk|fclk|mclk" gpurun_out/power_busy_$DIV.txt | head -24
