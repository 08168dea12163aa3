"""faasbal -- MI355X-native push balancer for Distributed-FaaS.

The hot path of ``PushDispatcher.start_heartbeat`` (reference
task_dispatcher.py:324-419) as CDNA4 HIP kernels behind a C ABI
(include/faasbal.h).  ``GpuBalancer`` is the tick-level handle;
``GpuPushDispatcher`` is the drop-in for the reference dispatcher class.
"""
from ._lib import FaasbalError  # noqa: F401
from .balancer import GpuBalancer  # noqa: F401
from .dispatcher import GpuPushDispatcher  # noqa: F401
from . import synth  # noqa: F401

EV_REGISTER, EV_RECONNECT, EV_HEARTBEAT, EV_RESULT, EV_OTHER = 0, 1, 2, 3, 4
