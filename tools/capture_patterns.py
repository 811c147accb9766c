"""Debug aid: which fork / join patterns of HIP streams survive a hipGraph capture on
this ROCm.  Each pattern runs in its own process (a bad one ends in a segmentation
fault inside hipStreamEndCapture):  python tools/capture_patterns.py [pattern]"""
import subprocess
import sys

import torch

# a pattern: list of ops over streams O (capture origin), S, P, Q:
#   "k X"    a kernel on X;   "w X Y"  X waits on Y's pending work (X.wait_stream(Y))
PATTERNS = {
    "fork_join": "w S O|k S|w O S",
    "nested": "w S O|w P S|k P|w S P|k S|w O S",
    "nested_back": "w S O|w P S|k P|w S P|k S|w P S|k P|w S P|w O S",
    "nested_origin_join": "w S O|w P S|k P|w S P|k S|w O S|w P O|k P|w O P",
    "sibling_mutual": "w S O|w P O|k S|k P|w S P|k S|w P S|k P|w O S|w O P",
    "sibling_oneway": "w S O|w P O|k P|w S P|k S|w O S|w O P",
    "sibling_back": "w S O|w P O|k P|w S P|k S|w P S|k P|w O S|w O P",
    "child_waits_origin": "w S O|w P S|k P|w S P|k O|w P O|k P|w O P|w O S",
    "design": "w S O|w P S|w Q O|k P|k Q|k S|w S P|k S|w O Q|k O|w Q O|k Q|w P S|k P|w O P|w O Q|w O S",
}


def run(pattern):
    dev = torch.device("cuda:0")
    x = torch.zeros(1024, device=dev)
    names = {"S": torch.cuda.Stream(dev), "P": torch.cuda.Stream(dev),
             "Q": torch.cuda.Stream(dev)}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        names["O"] = torch.cuda.current_stream(dev)
        for op in pattern.split("|"):
            f = op.split()
            if f[0] == "k":
                with torch.cuda.stream(names[f[1]]):
                    x.add_(1)
            else:
                names[f[1]].wait_stream(names[f[2]])
    g.replay()
    torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(PATTERNS[sys.argv[1]])
        sys.exit(0)
    for name in PATTERNS:
        rc = subprocess.call([sys.executable, __file__, name], stderr=subprocess.DEVNULL)
        print(f"{name:22s} rc={rc}", flush=True)
