"""Core IR: dtypes, devices, proxies, symbols, traces, prims, frontend, transforms."""
