def cached_path(*a, **k):
    raise RuntimeError("no network")
