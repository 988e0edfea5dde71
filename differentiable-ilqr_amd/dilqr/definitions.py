"""Value types of the reference API (definitions.py:3-4; defaults as set at
mpc_explicit.py:24-25)."""
from collections import namedtuple

QuadCost = namedtuple("QuadCost", "C c")
LinDx = namedtuple("LinDx", "F f")
QuadCost.__new__.__defaults__ = (None,) * len(QuadCost._fields)
LinDx.__new__.__defaults__ = (None,) * len(LinDx._fields)
