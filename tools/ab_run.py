#!/usr/bin/env python3
"""A/B helper: run another tool (tools/<name>.py's main) against an alternate build of the
engine library, e.g. the library before a kernel change:
    python tools/ab_run.py tools/ab/libsgx_base.so prof_configs --configs terasort:1024
"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    lib, tool, rest = sys.argv[1], sys.argv[2], sys.argv[3:]
    import sparkucx_amd._lib as L

    L.LIB_PATH = os.path.abspath(lib)
    L.ALLOW_MISSING = True
    sys.argv = [tool + ".py"] + rest
    importlib.import_module(tool).main()


if __name__ == "__main__":
    main()
