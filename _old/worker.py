"""Worker entry point — reference ``mnist_*/worker.py``.

Launch one per GPU (``run.sh`` does it).  Parameter-server roles are co-located in
these processes (PS p on rank p % W), so this one script covers the reference's
``worker.py`` *and* ``parameter_server.py`` ranks.  ``-np N`` is accepted for
command-line compatibility with the reference.
"""
import sys

from ddl_amd.parallel.launch import main

if __name__ == "__main__":
    main(sys.argv[1:])
