"""Reference ``detect_scripts`` package: the hot-path detection helpers (demo I/O is out of scope)."""
