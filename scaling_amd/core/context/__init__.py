from .context import BaseContext, BaseContextGeneric, ContextState, DeterminedBaseContext

__all__ = ["BaseContext", "BaseContextGeneric", "ContextState", "DeterminedBaseContext"]
