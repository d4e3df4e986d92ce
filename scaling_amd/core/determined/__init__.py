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


def determined_profiler_from_ctx(ctx: Any, dir_: Optional[str] = None, global_rank: int = 0) -> Any:
    if det is None or ctx is None:
        return None
    return None
