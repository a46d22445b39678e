"""Import harness for the read-only pyABC 0.10.5 reference (THIS container only).

Test infrastructure, never shipped or imported by the product: it lets
``make_golden.py`` import ``/root/reference/pyabc`` to produce golden vectors.
Optional dependencies that are absent from the image are stubbed, and the
pandas>=2 ``DataFrame.pivot`` positional-argument break used at
``pyabc/storage/history.py:307`` is shimmed.
"""
import sys
import types


class _Bar:
    def __init__(self, it=None, total=None, enable=False, keep=False, **kw):
        self.it = it

    def __iter__(self):
        return iter(self.it)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def inc(self, *a, **k):
        pass


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _Dummy:
    def __init__(self, *a, **k):
        raise RuntimeError("stubbed dependency")


class _GitErr(Exception):
    pass


class _Repo:
    def __init__(self, *a, **k):
        raise _GitErr("stubbed git")


_exc = types.SimpleNamespace(NoSuchPathError=_GitErr,
                             InvalidGitRepositoryError=_GitErr)
_mod("jabbar", jabbar=_Bar)
_mod("redis", StrictRedis=_Dummy)
_mod("distributed", Client=_Dummy)
_mod("git", Repo=_Repo, exc=_exc, InvalidGitRepositoryError=_GitErr,
     NoSuchPathError=_GitErr)
_mod("flask_bootstrap", Bootstrap=_Dummy)
_mod("feather")

import pandas as _pd  # noqa: E402

_orig_pivot = _pd.DataFrame.pivot


def _pivot(self, *args, **kwargs):
    for n, a in zip(["index", "columns", "values"], args):
        kwargs[n] = a
    return _orig_pivot(self, **kwargs)


_pd.DataFrame.pivot = _pivot
