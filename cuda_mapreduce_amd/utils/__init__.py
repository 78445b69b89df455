"""Small helpers: size parsing and formatting."""
from .sizes import fmt_bytes, parse_size  # noqa: F401
