"""Console progress bar and duration formatting.

Behavioural twin of the reference's xlua-style bar (src/utils.py:45-124): a
65-column ``[====>....]`` bar, per-step and total time, a caller message and a
``cur/total`` counter.  Fixes quirk A9: the reference reads the terminal width
with ``os.popen('stty size')`` AT IMPORT and crashes without a TTY; here the
width comes from :func:`shutil.get_terminal_size` (falls back to 80 columns)
and, when stdout is not a TTY, only the final line of each bar is printed so
logs stay readable.
"""
from __future__ import annotations

import shutil
import sys
import time
from typing import Optional, TextIO

BAR_COLS = 65
_UNITS = (("D", 86400.0), ("h", 3600.0), ("m", 60.0), ("s", 1.0), ("ms", 1e-3))


def format_time(seconds: float) -> str:
    """Two most significant non-zero units, e.g. ``1m5s``, ``3s120ms``, ``0ms``."""
    out = []
    rem = max(0.0, float(seconds))
    for suffix, size in _UNITS:
        q = int(rem / size + 1e-9)
        rem -= q * size
        if q > 0:
            out.append(f"{q}{suffix}")
            if len(out) == 2:
                break
    return "".join(out) or "0ms"


class ProgressBar:
    def __init__(self, stream: Optional[TextIO] = None, width: Optional[int] = None):
        self.stream = stream or sys.stdout
        self.width = width or shutil.get_terminal_size((80, 24)).columns
        self.t_begin = self.t_last = time.time()

    def update(self, current: int, total: int, msg: Optional[str] = None) -> str:
        now = time.time()
        if current == 0:
            self.t_begin = self.t_last = now
        step, tot = now - self.t_last, now - self.t_begin
        self.t_last = now
        done = int(BAR_COLS * current / max(total, 1))
        bar = " [" + "=" * done + ">" + "." * max(0, BAR_COLS - done - 1) + "]"
        text = f"  Step: {format_time(step)} | Tot: {format_time(tot)}"
        if msg:
            text += " | " + msg
        line = f"{bar}{text} {current + 1}/{total}"
        last = current >= total - 1
        tty = getattr(self.stream, "isatty", lambda: False)()
        if tty:
            self.stream.write("\r" + line.ljust(self.width - 1)[: max(self.width - 1, len(line))])
            if last:
                self.stream.write("\n")
            self.stream.flush()
        elif last:
            self.stream.write(line + "\n")
            self.stream.flush()
        return line


_default: Optional[ProgressBar] = None


def progress_bar(current: int, total: int, msg: Optional[str] = None) -> str:
    """Module-level convenience with the reference's call signature."""
    global _default
    if _default is None:
        _default = ProgressBar()
    return _default.update(current, total, msg)
