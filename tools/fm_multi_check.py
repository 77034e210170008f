import sys, os
sys.path.insert(0, os.getcwd())
import torch, bench
from gsdr_amd.signals import lowpass_taps
dev = torch.device("cuda", 0)
taps = torch.from_numpy(lowpass_taps(127, 0.1)).to(dev)
print(bench.fm_multi_gpu(torch, dev, taps, 0, 1, 50))
