#!/usr/bin/env python
"""Reference-compatible launcher: ``python microbeast.py --exp_name X [--test]``.

Multi-GPU: ``torchrun --nproc-per-node 8 --master-addr 127.0.0.1 microbeast.py ...``.
"""
import sys

from microbeast_amd.cli import main

if __name__ == "__main__":
    sys.exit(main())
