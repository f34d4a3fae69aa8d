"""Parameter-server entry point — reference ``mnist_*/parameter_server.py``.

On MI355X the PS shards live inside the GPU worker processes (RCCL cannot put two ranks
of one communicator on one GPU; a PS with no GPU would drag every gradient through host
memory).  ``ParameterServer`` is importable from here for API parity; running this file
behaves like ``worker.py`` with ``--num-ps`` taken from ``-np``.
"""
import sys

from ddl_amd.parallel.ps import ParameterServer  # noqa: F401  (API parity)
from ddl_amd.parallel.launch import main

if __name__ == "__main__":
    argv = sys.argv[1:]
    if "-np" in argv and "--num-ps" not in argv:
        i = argv.index("-np")
        argv = argv[:i] + ["--num-ps", argv[i + 1]] + argv[i + 2:]
    main(argv)
