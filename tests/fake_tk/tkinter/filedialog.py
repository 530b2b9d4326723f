SAVE_PATHS = []
OPEN_PATHS = []


def asksaveasfilename(**kw):
    return SAVE_PATHS.pop(0) if SAVE_PATHS else ""


def askopenfilename(**kw):
    return OPEN_PATHS.pop(0) if OPEN_PATHS else ""
