"""Runs scripts/graph_rccl_probe.hip (built as wiser_amd/_lib/libgraph_probe.so)
on torch's HIP runtime and RCCL: capture modes x sizes.  Usage: MODE N PAIRS"""
import ctypes
import os
import sys

import torch  # noqa: F401  (maps torch's libamdhip64 / librccl first)

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "wiser_amd", "_lib",
                               "libgraph_probe.so"))
mode, n, pairs = (int(x) for x in sys.argv[1:4])
rc = lib.probe(mode, n, pairs)
sys.stdout.flush()
sys.exit(rc)
