"""GPU choice for `pixpath.cli` processes started by the reference's pool.

The reference runs every builder string through ``ParallelRunner`` --
``Pool(max_parallel).starmap(subprocess.run(cmd, shell=True))``
(lib/cmd_utils.py:93-101) -- so a command cannot know its worker index, and a
process-id rule (pid % n_gpus) lets several workers land on one GPU while
others idle.  Instead every pixpath process takes the lowest free *slot*: an
exclusive ``flock`` on ``<dir>/gpu-slot-<i>.lock``, held for the life of the
process.  Slot i maps to device i % n_gpus, so the first n processes get n
different GPUs, the next n the second slot on each, and so on -- balanced and
deterministic for any pool size.

Order of precedence in ``choose_device``: PIXPATH_DEVICE (explicit), then
LOCAL_RANK (a torch.distributed / pixpath.batch launcher), then a slot.
"""
import fcntl
import os
import tempfile

_held = []


def slot_dir():
    return os.environ.get("PIXPATH_SLOT_DIR", os.path.join(tempfile.gettempdir(), "pixpath-slots-%d" % os.getuid()))


def acquire_slot(n_devices, max_levels=64):
    """Lock the lowest free slot; return (slot, device).  The lock is released
    when the process exits (or by release_slots())."""
    if n_devices <= 0:
        raise ValueError("no devices")
    d = slot_dir()
    os.makedirs(d, exist_ok=True)
    for i in range(n_devices * max_levels):
        fh = open(os.path.join(d, "gpu-slot-%d.lock" % i), "a")
        try:
            fcntl.flock(fh, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            fh.close()
            continue
        _held.append(fh)
        return i, i % n_devices
    raise RuntimeError("pixpath: more than %d processes per GPU" % max_levels)


def release_slots():
    while _held:
        fh = _held.pop()
        fcntl.flock(fh, fcntl.LOCK_UN)
        fh.close()


def choose_device(n_devices):
    d = os.environ.get("PIXPATH_DEVICE")
    if d is not None:
        return int(d)
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None:
        return int(lr) % n_devices
    return acquire_slot(n_devices)[1]


if __name__ == "__main__":  # used by tests: print the device a process would get, hold it briefly
    import sys
    import time
    print(acquire_slot(int(sys.argv[1]))[1], flush=True)
    time.sleep(float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
