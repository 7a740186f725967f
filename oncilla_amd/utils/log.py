"""Python-side logging gated like the native side: on when OCM_VERBOSE exists."""
from __future__ import annotations

import os
import sys
import time


def verbose() -> bool:
    return "OCM_VERBOSE" in os.environ


def log(msg: str) -> None:
    if verbose():
        print(f"[ocm-py {time.time():.6f} pid:{os.getpid()}] {msg}", file=sys.stderr, flush=True)
