"""Wire codec of the push dispatcher's ZMQ messages.

Same format as the reference (``helper_functions.py:5-9``): the object is
pickled with ``dill`` and base64-encoded (with the ``codecs`` line breaks), and
sent as UTF-8 bytes.  Workers running the reference's ``push_worker.py`` read
and write exactly this, so the GPU dispatcher is wire-compatible with them.
``dill`` is part of the reference's environment; plain ``pickle`` reads and
writes the same bytes for the dict messages the dispatcher exchanges, and is
used only when ``dill`` is not importable.
"""
from __future__ import annotations

import codecs

try:  # the reference's serializer
    import dill as _pickler
except ImportError:  # pragma: no cover - dill ships with the reference's environment
    import pickle as _pickler


def serialize(obj) -> str:
    return codecs.encode(_pickler.dumps(obj), "base64").decode()


def deserialize(ser_obj: str):
    return _pickler.loads(codecs.decode(ser_obj.encode(), "base64"))
