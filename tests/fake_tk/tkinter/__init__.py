"""Headless stand-in for ``tkinter`` (not installed here): widgets record their options and
children, ``Button.invoke()`` runs the command, ``Entry`` holds scripted text.  Lets the
reference ``lms_gui_final.py`` run UNCHANGED in tests (SURVEY.md §4.3 "GUI compat")."""
import threading

_lock = threading.RLock()
REGISTRY = []


class Widget:
    def __init__(self, master=None, *args, **kw):
        self.master = master
        self.kw = dict(kw)
        self.children = []
        self.destroyed = False
        with _lock:
            REGISTRY.append(self)
            if master is not None:
                master.children.append(self)

    # geometry managers / config
    def grid(self, *a, **k): pass
    def pack(self, *a, **k): pass
    def place(self, *a, **k): pass
    def grid_rowconfigure(self, *a, **k): pass
    def grid_columnconfigure(self, *a, **k): pass
    def rowconfigure(self, *a, **k): pass
    def columnconfigure(self, *a, **k): pass
    def bind(self, *a, **k): pass
    def focus_set(self): pass
    def update(self): pass
    def update_idletasks(self): pass

    def config(self, **kw):
        self.kw.update(kw)

    configure = config

    def cget(self, key):
        return self.kw.get(key)

    def destroy(self):
        with _lock:
            self.destroyed = True
            for c in list(self.children):
                c.destroy()
            if self.master is not None and self in self.master.children:
                self.master.children.remove(self)

    def winfo_exists(self):
        return not self.destroyed

    def winfo_children(self):
        with _lock:
            return list(self.children)

    def after(self, ms, func=None, *args):
        return "after#0"  # animations are not run headless

    def after_cancel(self, _id): pass


class Tk(Widget):
    def __init__(self, *a, **k):
        super().__init__(None)
        self._title = ""

    def title(self, t=None):
        if t is not None:
            self._title = t
        return self._title

    def geometry(self, *a): pass
    def mainloop(self): pass
    def quit(self): pass
    def resizable(self, *a): pass


class Frame(Widget): pass
class Label(Widget): pass
class Toplevel(Widget): pass
class Canvas(Widget): pass
class Scrollbar(Widget): pass
class Listbox(Widget): pass


class Button(Widget):
    def invoke(self):
        cmd = self.kw.get("command")
        return cmd() if cmd else None


class Entry(Widget):
    def __init__(self, master=None, *a, **k):
        super().__init__(master, *a, **k)
        self.value = ""

    def get(self):
        return self.value

    def insert(self, index, s):
        self.value += str(s)

    def delete(self, first, last=None):
        self.value = ""


class Variable:
    def __init__(self, master=None, value=None, name=None):
        self._v = value

    def get(self):
        return self._v

    def set(self, v):
        self._v = v


class StringVar(Variable):
    def __init__(self, master=None, value="", name=None):
        super().__init__(master, value, name)


class IntVar(Variable):
    def __init__(self, master=None, value=0, name=None):
        super().__init__(master, value, name)


class Radiobutton(Widget):
    def invoke(self):
        self.kw["variable"].set(self.kw["value"])


class OptionMenu(Widget):
    def __init__(self, master, variable, value, *values, **kw):
        super().__init__(master, **kw)
        self.variable = variable
        self.values = [value, *values]


END = "end"
LEFT, RIGHT, TOP, BOTTOM, BOTH, X, Y = "left", "right", "top", "bottom", "both", "x", "y"
W, E, N, S = "w", "e", "n", "s"


def find_buttons(text):
    with _lock:
        return [w for w in REGISTRY if isinstance(w, Button) and not w.destroyed and w.kw.get("text") == text]
