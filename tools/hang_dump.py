"""Debug hook (SCALING_AMD_DEBUG_HOOKS=tools/hang_dump.py): after HANG_DUMP_S seconds (default 90) every thread's stack
goes to gpurun_out/hang.rank<r>.txt and the process exits -- for a run suspected to hang."""
import faulthandler
import os

os.makedirs("gpurun_out", exist_ok=True)
_f = open(f"gpurun_out/hang.rank{os.environ.get('RANK', '0')}.txt", "w")
faulthandler.dump_traceback_later(float(os.environ.get("HANG_DUMP_S", "90")), exit=True, file=_f)
