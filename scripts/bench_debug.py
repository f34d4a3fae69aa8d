#!/usr/bin/env python3
"""bench.py with a watchdog that dumps every thread's Python stack after 90 seconds and exits —
for locating a stall in a multi-process rehearsal."""
import faulthandler
import os
import runpy
import sys

faulthandler.dump_traceback_later(90.0, exit=True)
sys.argv[0] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
runpy.run_path(sys.argv[0], run_name="__main__")
