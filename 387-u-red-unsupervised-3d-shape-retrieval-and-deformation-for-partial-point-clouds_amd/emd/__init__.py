from .emd_module import emdModule as emd  # noqa: F401  (utils_v2/metrics/EMD/__init__.py:1)
