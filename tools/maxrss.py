"""Run a command as a child process and report its peak resident memory (RUSAGE_CHILDREN) on stderr."""
import resource
import subprocess
import sys
import time

t = time.time()
rc = subprocess.call(sys.argv[1:])
ru = resource.getrusage(resource.RUSAGE_CHILDREN)
sys.stderr.write(f"[maxrss] {ru.ru_maxrss / 1048576:.2f} GiB peak RSS, {time.time() - t:.1f} s, rc {rc}\n")
sys.exit(rc)
