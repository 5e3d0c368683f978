"""A small JSON-schema checker for the reference's window schemas (draft-07 subset they use:
type, properties, required, additionalProperties, items, anyOf). jsonschema is not installed.
Test infrastructure only."""

_TYPES = {"object": dict, "array": list, "string": str, "boolean": bool, "null": type(None)}


def _is(t, v):
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool)
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return isinstance(v, _TYPES[t])


def errors(schema, v, path="$"):
    """list of violations of `schema` by `v` (empty when it conforms)"""
    out = []
    if not isinstance(schema, dict):
        return out
    if "anyOf" in schema:
        if all(errors(s, v, path) for s in schema["anyOf"]):
            out.append(f"{path}: matches none of anyOf")
    t = schema.get("type")
    if t is not None:
        ts = t if isinstance(t, list) else [t]
        if not any(_is(x, v) for x in ts):
            return out + [f"{path}: {type(v).__name__} is not {t}"]
    if isinstance(v, dict):
        props = schema.get("properties", {})
        for k in schema.get("required", []):
            if k not in v:
                out.append(f"{path}: missing required '{k}'")
        for k, x in v.items():
            if k in props:
                out += errors(props[k], x, f"{path}.{k}")
            else:
                ap = schema.get("additionalProperties", True)
                if ap is False:
                    out.append(f"{path}: additional property '{k}'")
                elif isinstance(ap, dict):
                    out += errors(ap, x, f"{path}.{k}")
    if isinstance(v, list) and "items" in schema:
        it = schema["items"]
        if isinstance(it, list):
            for i, (s, x) in enumerate(zip(it, v)):
                out += errors(s, x, f"{path}[{i}]")
        else:
            for i, x in enumerate(v):
                out += errors(it, x, f"{path}[{i}]")
    return out
