"""Region-text loader and colour names -- replaces the reference's path_generation/utils.py.

``get_var_from_file`` (utils.py:29-35) ``exec``s the text; here the text is parsed with
``ast`` and only literal calls ``polygon([x, y], ...)``, ``ball(...)`` and ``square(...)`` are
accepted, so a data file cannot run code.  ``color2RGB`` maps the same single-letter / name
colours to RGB lists (utils.py:3-27)."""
import ast

_COLORS = {"k": [0, 0, 0], "black": [0, 0, 0], "b": [0, 0, 1], "blue": [0, 0, 1],
           "g": [0, 1, 0], "green": [0, 1, 0], "c": [0, 1, 1], "cyan": [0, 1, 1],
           "r": [1, 0, 0], "red": [1, 0, 0], "m": [1, 0, 1], "magenta": [1, 0, 1],
           "y": [1, 1, 0], "yellow": [1, 1, 0], "w": [1, 1, 1], "white": [1, 1, 1]}


def color2RGB(color):
    if not isinstance(color, str):
        return color
    return _COLORS.get(color.lower())


def _literal(node):
    return ast.literal_eval(node)


def parse_shapes_text(content, varname="vertices"):
    """Return {varname: [(kind, args, kwargs), ...]} from a D1-style text without executing it."""
    tree = ast.parse(content)
    found = {}
    for stmt in tree.body:
        if not (isinstance(stmt, ast.Assign) and len(stmt.targets) == 1
                and isinstance(stmt.targets[0], ast.Name)):
            raise ValueError("only 'name = [shape(...), ...]' assignments are allowed")
        value = stmt.value
        items = value.elts if isinstance(value, (ast.List, ast.Tuple)) else [value]
        shapes = []
        for it in items:
            if isinstance(it, ast.Call) and isinstance(it.func, ast.Name) \
                    and it.func.id in ("polygon", "ball", "square"):
                args = [_literal(a) for a in it.args]
                kwargs = {k.arg: _literal(k.value) for k in it.keywords}
                shapes.append((it.func.id, args, kwargs))
            else:
                shapes.append(("literal", [_literal(it)], {}))
        found[stmt.targets[0].id] = shapes
    return found


def get_var_from_file(filename, varname):
    from .ball import ball
    from .polygon import polygon
    from .square import square

    makers = {"polygon": polygon, "ball": ball, "square": square}
    with open(filename, "r") as f:
        content = f.read()
    parsed = parse_shapes_text(content, varname)
    if varname not in parsed:
        raise KeyError(varname)
    out = []
    for kind, args, kwargs in parsed[varname]:
        out.append(args[0] if kind == "literal" else makers[kind](*args, **kwargs))
    return out
