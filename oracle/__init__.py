"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/oracle.py). Imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product."""
from .oracle import *  # noqa: F401,F403
from .oracle import _act, build, lib  # noqa: F401
