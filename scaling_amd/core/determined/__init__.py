"""Optional Determined AI integration (reference ``core/determined/core.py`` and
``utils/determined_utils.py``).  ``determined`` is not part of the MI355X image, so everything here
degrades to no-ops unless the package is importable."""
from __future__ import annotations

import faulthandler
import sys
from contextlib import contextmanager
from typing import Any, Iterator, Optional

try:  # pragma: no cover - optional dependency
    import determined as det  # type: ignore
except ImportError:  # pragma: no cover
    det = None


def available() -> bool:
    return det is not None


@contextmanager
def init(distributed: Any = None, **kwargs: Any) -> Iterator[Any]:
    if det is None:
        raise RuntimeError("determined is not installed")
    with det.core.init(distributed=distributed, tensorboard_mode=det.core.TensorboardMode.MANUAL, **kwargs) as ctx:
        yield ctx


def maybe_periodic_stacktraces(debug_enabled: bool, period_s: int = 30) -> None:
    if debug_enabled:
        faulthandler.dump_traceback_later(period_s, repeat=True, file=sys.stderr)


def determined_profiler_from_ctx(ctx: Any, config_determined: Any = None, info: Any = None) -> Any:
    """Determined's ProfilerAgent for this trial (reference ``utils/determined_utils.py:29``).

    Returns None when ``determined`` is not installed or there is no cluster context; the trainer then
    skips ``update_batch_idx``.  ``config_determined`` provides ``profiling_interval()``,
    ``profiling_enabled()`` and ``profiling_sync_timings()`` (Determined's ExperimentConfig)."""
    if det is None or ctx is None or config_determined is None or info is None:
        return None
    begin_on_batch, end_after_batch = config_determined.profiling_interval()
    return det.profiler.ProfilerAgent(
        trial_id=str(ctx.train._trial_id), agent_id=info.agent_id, master_url=info.master_url,
        profiling_is_enabled=config_determined.profiling_enabled(), global_rank=ctx.distributed.get_rank(),
        local_rank=ctx.distributed.get_local_rank(), begin_on_batch=begin_on_batch, end_after_batch=end_after_batch,
        sync_timings=config_determined.profiling_sync_timings(),
    )
