"""Wire codec of the push dispatcher's ZMQ messages.

Same format as the reference (``helper_functions.py:5-9``): the object is
pickled with ``dill`` and base64-encoded (with the ``codecs`` line breaks), and
sent as UTF-8 bytes.  Workers running the reference's ``push_worker.py`` read
and write exactly this, so the GPU dispatcher is wire-compatible with them.

The dispatcher's own messages are plain data (dicts of strings and numbers).
For those, dill's pure-Python pickler writes exactly the bytes the C pickler
writes at dill's protocol, so ``serialize`` takes the C path for plain data
(≈9x faster per message) and dill for anything else (functions, classes);
``tests/test_dispatcher.py`` checks the bytes against dill's.  ``deserialize``
reads with the C unpickler and falls back to dill's for what it cannot read.
``dill`` is part of the reference's environment; plain ``pickle`` is used
alone only when ``dill`` is not importable.
"""
from __future__ import annotations

import codecs
import pickle

try:  # the reference's serializer
    import dill as _dill
    _PROTOCOL = _dill.settings["protocol"]
except ImportError:  # pragma: no cover - dill ships with the reference's environment
    _dill = None
    _PROTOCOL = pickle.DEFAULT_PROTOCOL

_SCALARS = (str, bytes, int, float, bool, type(None))


def _plain(obj, depth=0) -> bool:
    """Built-in data only (what the dispatcher and workers exchange as messages)."""
    t = type(obj)
    if t in _SCALARS:
        return True
    if depth > 8:
        return False
    if t is dict:
        return all(type(k) in _SCALARS and _plain(v, depth + 1) for k, v in obj.items())
    if t is list or t is tuple:
        return all(_plain(v, depth + 1) for v in obj)
    return False


def serialize(obj) -> str:
    if _dill is None or _plain(obj):
        data = pickle.dumps(obj, protocol=_PROTOCOL)
    else:
        data = _dill.dumps(obj)
    return codecs.encode(data, "base64").decode()


def deserialize(ser_obj: str):
    data = codecs.decode(ser_obj.encode(), "base64")
    try:
        return pickle.loads(data)
    except Exception:
        if _dill is None:
            raise
        return _dill.loads(data)
