"""Single-process trainer — reference ``mnist_sync/single.py`` (``Single(1, 100).train()``).

Runs the CNN on one MI355X through the HIP engine (or on the CPU through the torch
oracle when no GPU is present).  Prints the reference's lines:
``epoch: {} batch: {} accuracy: {}`` every 10 steps and ``final accuracy: {}``.
"""
import sys

from ddl_amd.parallel.launch import main

if __name__ == "__main__":
    main(["--mode", "single"] + sys.argv[1:], mode_default="single")
