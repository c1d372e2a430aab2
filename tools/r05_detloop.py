import os, sys, torch
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tests")]
import importlib
from __graft_entry__ import load_package
pkg = load_package()
import test_gpu_parity as T
dev = torch.device("cuda", 0)
bad = 0
for trial in range(4):
    try:
        T.test_dense_backward_bf16_deterministic(pkg, dev)
    except AssertionError as e:
        bad += 1
        print("FAIL", os.environ.get("PG_DIRECTGCN_LIB", "default").split("/")[-1], e.args[0] if e.args else e, flush=True)
print("lib", os.environ.get("PG_DIRECTGCN_LIB", "default").split("/")[-1], "failed trials", bad, "of 4", flush=True)
