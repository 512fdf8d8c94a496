import sys, os, time, json, argparse
sys.path.insert(0, os.getcwd())
import torch
import bench
ap = argparse.Namespace(steps=10, warmup=3, chunks=0, lda_pad=0, split_d=False, no_cpu_baseline=True, prefilled=False, dist=False, gpus=1)
dev = torch.device("cuda", 0)
def run(cfg):
    r = bench.run_config(ap, cfg, False, 1, 0, dev, False)
    return round(r["kernel_ms"], 4), round(r["ms_per_step"], 4)
print("c3 first", run("c3"), flush=True)
print("c2", run("c2"), flush=True)
print("c3 after c2", run("c3"), flush=True)
print("ns", run("ns"), flush=True)
print("c3 after ns", run("c3"), flush=True)
time.sleep(2.0)
print("c3 after ns + 2 s", run("c3"), flush=True)
print("ns", run("ns"), flush=True)
torch.cuda.synchronize(); time.sleep(0.5)
print("c3 after ns + 0.5 s", run("c3"), flush=True)
