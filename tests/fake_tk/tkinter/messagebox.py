import threading

LOG = []
_cv = threading.Condition()


def _rec(kind, title, message=None, **kw):
    with _cv:
        LOG.append((kind, title, message))
        _cv.notify_all()
    return True


def showinfo(title=None, message=None, **kw): return _rec("info", title, message)
def showerror(title=None, message=None, **kw): return _rec("error", title, message)
def showwarning(title=None, message=None, **kw): return _rec("warning", title, message)
def askyesno(title=None, message=None, **kw): return _rec("ask", title, message)


def wait_for(n, timeout=30.0):
    """Block until at least n dialogs were shown; returns the log."""
    import time
    end = time.time() + timeout
    with _cv:
        while len(LOG) < n and time.time() < end:
            _cv.wait(0.05)
        return list(LOG)
