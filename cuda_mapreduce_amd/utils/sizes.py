"""Human-readable sizes (same grammar as the CLI's --synthetic / --chunk-bytes)."""
_UNITS = {"": 1, "K": 1 << 10, "M": 1 << 20, "G": 1 << 30, "T": 1 << 40}


def parse_size(s: str) -> int:
    s = s.strip().upper().rstrip("B")
    unit = s[-1] if s and s[-1] in "KMGT" else ""
    return int(float(s[: len(s) - len(unit)]) * _UNITS[unit])


def fmt_bytes(n: float) -> str:
    for u in ("B", "KiB", "MiB", "GiB", "TiB"):
        if n < 1024 or u == "TiB":
            return f"{n:.1f} {u}" if u != "B" else f"{int(n)} B"
        n /= 1024
    return str(n)
