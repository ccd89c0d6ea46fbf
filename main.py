#!/usr/bin/env python
"""Reference-compatible standalone trainer: `python3 main.py [--lr LR] [-r] [-a NAME]`
(the reference's src/main.py train(epoch)/test(epoch) mode).  See fedmi.cli.train.
"""
import sys

from fedmi.cli.train import main

if __name__ == "__main__":
    sys.exit(main())
