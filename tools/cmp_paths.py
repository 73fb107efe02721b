import sys, time, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/ee274_convexcaldera_llm_quantization_amd")
import bench
from ee274_convexcaldera_llm_quantization_amd import api
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
qp = bench.make_params(); ep = EngineParams.from_caldera_params(qp)
dev = torch.device("cuda", 0)
B = int(sys.argv[1])
W = bench.synth_batch(B, 0, dev)
def t(fn, n=2):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1000
print("engine", t(lambda: CalderaEngine(ep).run(W, None)))
print("api   ", t(lambda: api.caldera_batch(qp, W, None, device=dev)))
print("engine", t(lambda: CalderaEngine(ep).run(W, None)))
