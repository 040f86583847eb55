"""Fortran namelist input for flux_calculator.nml (flux_calculator.F90:55-129, 174-177) and
the bias-correction group (bias_corrections.F90:52, 120-150).

`read_namelist(text, group, spec)` applies a group to the declared defaults with the
semantics of a Fortran `READ(unit, nml=group)`:
  * `name = v1, v2, ...` fills the array from its first element in array-element
    (column-major) order; `name(i,j,k) = ...` starts at that element; `name(1,2,:)` or
    `name(1,2:4,1)` fill the section's elements in column-major order;
  * `r*value` repeats, `r*` and empty values between commas are nulls (element unchanged);
  * CHARACTER(len=L) values are truncated / blank-padded to L (kept here without the
    trailing blanks, as every use in the reference TRIMs them or compares to 'none');
  * logicals accept T/F/.TRUE./.FALSE. in any case and any text after the letter;
  * reals accept d/D exponents; `!` starts a comment outside quotes;
  * an unknown variable or too many values raise ValueError, as the Fortran READ fails.
The group ends at `/` or `&end`.  Only the first occurrence of the group is read, like
one READ statement.
"""
import re

import numpy as np

from .basic import MAX_BOTTOM_MODELS, MAX_SURFACE_TYPES

MAX_TASKS_PER_MODEL = 1000  # basic:29
MAX_VARS = 100  # basic:30


class Var:
    """One namelist object: kind in {'int', 'real', 'logical', 'char'}, Fortran shape."""

    def __init__(self, kind, shape=(), default=None, length=None):
        self.kind, self.shape, self.default, self.length = kind, tuple(shape), default, length

    def new(self):
        if not self.shape:
            return self.default
        a = np.empty(self.shape, dtype=object)
        a.fill(self.default)
        return a


B, S, V = MAX_BOTTOM_MODELS, MAX_SURFACE_TYPES, MAX_VARS

# flux_calculator.F90:55-107 (+ verbosity_level, basic:74-79, default STANDARD = 1)
INPUT_SPEC = {
    "timestep": Var("int", (), 0),
    "num_timesteps": Var("int", (), 0),
    "verbosity_level": Var("int", (), 1),
    "name_atmos_model": Var("char", (), "", 50),
    "name_bottom_model": Var("char", (B,), "", 50),
    "letter_bottom_model": Var("char", (B,), "", 1),
    "num_tasks_per_model": Var("int", (B,), 0),
    "num_t_grid_cells": Var("int", (B, MAX_TASKS_PER_MODEL), 0),
    "num_u_grid_cells": Var("int", (B, MAX_TASKS_PER_MODEL), 0),
    "num_v_grid_cells": Var("int", (B, MAX_TASKS_PER_MODEL), 0),
    **{f"name_bottom_var_{g}": Var("char", (B, S, V), "none", 4) for g in "tuv"},
    **{f"name_atmos_var_{g}": Var("char", (V,), "none", 4) for g in "tuv"},
    **{f"name_send_{g}": Var("char", (V,), "none", 4) for g in "tuv"},
    **{f"send_to_atmos_{g}": Var("logical", (V,), True) for g in "tuv"},
    **{f"send_to_bottom_{g}": Var("logical", (B, V), True) for g in "tuv"},
    **{f"send_uniform_{g}": Var("logical", (B, V), False) for g in "tuv"},
    **{f"regrid_{k}": Var("char", (B, S, V), "none", 4) for k in ("u_to_t", "v_to_t", "t_to_u", "t_to_v")},
    **{f"val_bottom_var_{g}": Var("real", (B, S, V), -1.0e20) for g in "tuv"},
    **{f"val_atmos_var_{g}": Var("real", (V,), -1.0e20) for g in "tuv"},
    **{f"val_flux_{g}": Var("real", (V,), 0.0) for g in "tuv"},
    **{f"which_spec_vapor_surface_{g}": Var("char", (B, S), "none", 20) for g in "tuv"},
    **{k: Var("char", (B, S), "none", 20) for k in (
        "which_flux_mass_evap", "which_flux_heat_latent", "which_flux_heat_sensible",
        "which_flux_momentum", "which_flux_radiation_blackbody")},
}

# bias_corrections.F90:28-33, 52 (E_N_CORRECTIONS = 1)
CORRECTIONSCTL_SPEC = {
    "init_date": Var("int", (), 0),
    "lcorrections": Var("logical", (1,), False),
}

# ------------------------------------------------------------------------------ lexer

_NAME = re.compile(r"[A-Za-z][A-Za-z0-9_]*")


def _strip_comments(text):
    out, q = [], None
    for line in text.splitlines():
        buf = []
        for c in line:
            if q:
                buf.append(c)
                if c == q:
                    q = None
            elif c in "'\"":
                q = c
                buf.append(c)
            elif c == "!":
                break
            else:
                buf.append(c)
        out.append("".join(buf))
        # a string may not span lines in this reader (the reference namelists never do)
        q = None
    return "\n".join(out)


class _Lexer:
    def __init__(self, text):
        self.t = text
        self.i = 0

    def skip_ws(self):
        while self.i < len(self.t) and self.t[self.i] in " \t\r\n":
            self.i += 1

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else ""

    def at_end_of_group(self):
        self.skip_ws()
        if self.peek() == "/":
            return True
        return self.t[self.i:self.i + 4].lower() in ("&end", "$end")

    def assignment_ahead(self):
        """An object name (with optional subscripts) followed by '='."""
        m = _NAME.match(self.t, self.i)
        if not m:
            return None
        j = m.end()
        while j < len(self.t) and self.t[j] in " \t\r\n":
            j += 1
        sub = None
        if j < len(self.t) and self.t[j] == "(":
            k = self.t.find(")", j)
            if k < 0:
                return None
            sub = self.t[j + 1:k]
            j = k + 1
            while j < len(self.t) and self.t[j] in " \t\r\n":
                j += 1
        if j < len(self.t) and self.t[j] == "=":
            return m.group(0), sub, j + 1
        return None

    def value_token(self):
        """One value: a quoted string (optionally after r*), or a run up to a separator."""
        start = self.i
        buf = []
        while self.i < len(self.t):
            c = self.t[self.i]
            if c in "'\"":
                q = c
                self.i += 1
                s = []
                while self.i < len(self.t):
                    if self.t[self.i] == q:
                        if self.i + 1 < len(self.t) and self.t[self.i + 1] == q:
                            s.append(q)
                            self.i += 2
                            continue
                        self.i += 1
                        break
                    s.append(self.t[self.i])
                    self.i += 1
                else:
                    raise ValueError(f"unterminated string at offset {start}")
                buf.append(("q", "".join(s)))
                continue
            if c in " \t\r\n,/":
                break
            buf.append(("c", c))
            self.i += 1
        return buf


def _decode(tok):
    """(repeat, raw-or-None, quoted) from the token parts."""
    text = "".join(v if k == "c" else "" for k, v in tok)
    quoted = [v for k, v in tok if k == "q"]
    m = re.match(r"^(\d+)\*", text)
    rep = 1
    if m:
        rep = int(m.group(1))
        text = text[m.end():]
    if quoted:
        if text:
            raise ValueError(f"malformed value {''.join(v for _, v in tok)!r}")
        return rep, quoted[0], True
    if text == "":
        return rep, None, False  # r* : r nulls
    return rep, text, False


def _convert(var, raw, quoted, name):
    if var.kind == "char":
        return raw[: var.length] if var.length else raw
    if quoted:
        raise ValueError(f"{name}: character value {raw!r} for a {var.kind} variable")
    if var.kind == "int":
        try:
            return int(raw)
        except ValueError:
            raise ValueError(f"{name}: bad integer {raw!r}") from None
    if var.kind == "real":
        try:
            return float(raw.replace("d", "e").replace("D", "e"))
        except ValueError:
            raise ValueError(f"{name}: bad real {raw!r}") from None
    s = raw.lower().lstrip(".")
    if s[:1] == "t":
        return True
    if s[:1] == "f":
        return False
    raise ValueError(f"{name}: bad logical {raw!r}")


def _colmajor(shape):
    """Element tuples (0-based) in array-element order (first index fastest)."""
    for rev in np.ndindex(*reversed(shape)):
        yield tuple(reversed(rev))


def _targets(var, sub, name):
    """Element sequence assigned by `name(sub) = ...` (None: the whole array / scalar)."""
    if not var.shape:
        if sub is not None:
            raise ValueError(f"{name} is a scalar")
        return [None]
    if sub is None:
        return list(_colmajor(var.shape))
    parts = [p.strip() for p in sub.split(",")]
    if len(parts) != len(var.shape):
        raise ValueError(f"{name}({sub}): rank {len(var.shape)} expected")
    ranges, scalar = [], True
    for p, n in zip(parts, var.shape):
        if ":" in p:
            scalar = False
            lo, hi = (p.split(":") + [""])[:2]
            r = range(int(lo) - 1 if lo.strip() else 0, int(hi) if hi.strip() else n)
        else:
            r = range(int(p) - 1, int(p))
        if len(r) and (r.start < 0 or r.stop > n):
            raise ValueError(f"{name}({sub}): subscript out of bounds 1..{n}")
        ranges.append(r)
    if scalar:  # start here, continue through the rest of the array in element order
        start = tuple(r.start for r in ranges)
        seq = list(_colmajor(var.shape))
        return seq[seq.index(start):]
    shape = [len(r) for r in ranges]
    return [tuple(r[i] for r, i in zip(ranges, idx)) for idx in _colmajor(shape)]


def read_namelist(text, group, spec, values=None):
    """Apply the first `&group ... /` of `text` to the defaults of `spec` (or to `values`).
    Returns {name: scalar or numpy object array of the declared Fortran shape}.  A missing
    group raises ValueError (the Fortran READ hits end of file)."""
    vals = values if values is not None else {k: v.new() for k, v in spec.items()}
    text = _strip_comments(text)
    m = re.search(r"[&$]" + re.escape(group) + r"\b", text, flags=re.IGNORECASE)
    if not m:
        raise ValueError(f"namelist group &{group} not found")
    lx = _Lexer(text)
    lx.i = m.end()
    while True:
        if lx.at_end_of_group():
            break
        if lx.i >= len(lx.t):
            raise ValueError(f"namelist group &{group} is not terminated")
        a = lx.assignment_ahead()
        if a is None:
            raise ValueError(f"&{group}: expected 'name =' at {lx.t[lx.i:lx.i + 30]!r}")
        name, sub, lx.i = a[0].lower(), a[1], a[2]
        if name not in spec:
            raise ValueError(f"&{group}: unknown variable {a[0]!r}")
        var = spec[name]
        targets = _targets(var, sub, name)
        k = 0  # position in targets
        expect = True  # at the start and after a comma: a comma here is a null value
        while True:
            lx.skip_ws()
            if lx.peek() == "" or lx.at_end_of_group() or lx.assignment_ahead():
                break
            if lx.peek() == ",":
                lx.i += 1
                if expect:
                    k += 1
                expect = True
                continue
            rep, raw, quoted = _decode(lx.value_token())
            expect = False
            if raw is None:
                k += rep
                continue
            v = _convert(var, raw, quoted, name)
            for _ in range(rep):
                if k >= len(targets):
                    raise ValueError(f"&{group}: too many values for {name}")
                if targets[k] is None:
                    vals[name] = v
                else:
                    vals[name][targets[k]] = v
                k += 1
    return vals


def read_input(text):
    """flux_calculator.nml &input (flux_calculator.F90:174-177)."""
    return read_namelist(text, "input", INPUT_SPEC)


def read_correctionsctl(text):
    """flux_calculator.nml &correctionsctl (bias_corrections.F90:120-150)."""
    return read_namelist(text, "correctionsctl", CORRECTIONSCTL_SPEC)


__all__ = ["Var", "INPUT_SPEC", "CORRECTIONSCTL_SPEC", "MAX_TASKS_PER_MODEL", "MAX_VARS",
           "read_namelist", "read_input", "read_correctionsctl"]
