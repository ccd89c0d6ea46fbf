#!/usr/bin/env python
"""Reference-compatible entry point: `python3 client.py ...` (src/client.py of the reference).

Thin launcher for :mod:`fedmi.cli.client`; every reference flag is accepted.
"""
import sys

from fedmi.cli.client import main

if __name__ == "__main__":
    sys.exit(main())
