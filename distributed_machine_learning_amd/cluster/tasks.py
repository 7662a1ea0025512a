"""Fire-and-forget asyncio tasks that cannot be garbage-collected mid-flight.

An event loop holds only weak references to its tasks: a task that nothing else
references (``loop.create_task(coro)`` with the result dropped) can be destroyed
by the cyclic garbage collector while it is still pending ("Task was destroyed
but it is pending!") - a SWIM detector loop or a message reply that silently
never runs. ``spawn`` keeps a strong reference until the task finishes.
"""
from __future__ import annotations

import asyncio
from typing import Coroutine, Optional, Set

_live: Set[asyncio.Task] = set()


def spawn(coro: Coroutine, loop: Optional[asyncio.AbstractEventLoop] = None) -> asyncio.Task:
    """Schedule ``coro`` on ``loop`` (default: the running loop) and keep the task
    alive until it is done. Call from the loop's thread."""
    task = (loop or asyncio.get_running_loop()).create_task(coro)
    _live.add(task)
    task.add_done_callback(_live.discard)
    return task
