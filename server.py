#!/usr/bin/env python
"""Reference-compatible entry point: `python3 server.py ...` (src/server.py of the reference).

Thin launcher for :mod:`fedmi.cli.server`; every reference flag is accepted.
"""
import sys

from fedmi.cli.server import main

if __name__ == "__main__":
    sys.exit(main())
