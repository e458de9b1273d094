"""cProfile of BASELINE config 1's host round through the drop-in (bench.c1_host_round) on the GPU box:
where the host time of a tiny-model round goes.  usage: python tools/c1_profile.py"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench

    dev = torch.device("cuda:0")
    print(bench.c1_host_round(dev, 0, rounds=20))
    pr = cProfile.Profile()
    pr.enable()
    bench.c1_host_round(dev, 0, rounds=200)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
