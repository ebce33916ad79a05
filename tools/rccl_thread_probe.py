"""Run tools/librccl_thread_probe.so's modes A-D (see the .cpp), each in its own
process after `import torch`, against torch's RCCL and /opt/rocm's."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if len(sys.argv) == 3:
    import ctypes

    import torch  # noqa: F401  (torch's HIP runtime and RCCL first, as in bench.py)

    L = ctypes.CDLL(os.path.join(HERE, "librccl_thread_probe.so"))
    sys.exit(L.rccl_thread_probe(sys.argv[1].encode(), ctypes.c_char(sys.argv[2].encode())))
import torch

libs = {"torch": os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"),
        "rocm": "/opt/rocm/lib/librccl.so.1"}
for name, path in libs.items():
    for mode in "DABC":
        p = subprocess.run(["timeout", "-k", "5", "60", sys.executable, __file__, path, mode], capture_output=True,
                           text=True)
        lines = [ln for ln in p.stderr.splitlines() if ln.startswith("[")]
        print(f"== {name} mode {mode}: rc {p.returncode}", flush=True)
        for ln in lines:
            print("   " + ln, flush=True)
        if p.returncode:
            print("   stderr tail: " + " | ".join(p.stderr.splitlines()[-4:])[-600:], flush=True)
