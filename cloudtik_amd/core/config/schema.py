"""A dependency-free JSON-Schema (draft-07 subset) validator for cluster / runtime /
workspace configs (the reference validates with ``jsonschema`` against
``python/cloudtik/schema/*.json``; that package is not part of this image).

Supported keywords: type (incl. unions), properties, required, additionalProperties
(bool or schema), patternProperties, items, minItems, maxItems, enum, const, minimum,
maximum, exclusiveMinimum, minLength, maxLength, pattern, anyOf, oneOf, allOf, not,
$ref (local ``#/definitions/...``), default (ignored for validation).
"""
from __future__ import annotations

import re
from typing import Any, List


class ValidationError(ValueError):
    def __init__(self, message: str, path: List[str]):
        self.path = list(path)
        loc = "/".join(str(p) for p in path) or "<root>"
        super().__init__(f"{loc}: {message}")
        self.message = message


_TYPES = {
    "object": dict, "array": list, "string": str, "boolean": bool,
    "null": type(None),
}


def _is_type(v, t):
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool)
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return isinstance(v, _TYPES[t])


def _resolve(root, ref):
    if not ref.startswith("#/"):
        raise ValidationError(f"unsupported $ref {ref}", [])
    node = root
    for part in ref[2:].split("/"):
        node = node[part]
    return node


def validate(instance: Any, schema: dict, root: dict = None, path=None):
    root = root if root is not None else schema
    path = path or []
    if schema is True or schema == {}:
        return
    if schema is False:
        raise ValidationError("not allowed", path)
    if "$ref" in schema:
        validate(instance, _resolve(root, schema["$ref"]), root, path)
    t = schema.get("type")
    if t is not None:
        ts = t if isinstance(t, list) else [t]
        if not any(_is_type(instance, x) for x in ts):
            raise ValidationError(f"expected type {t}, got {type(instance).__name__}", path)
    if "enum" in schema and instance not in schema["enum"]:
        raise ValidationError(f"{instance!r} not one of {schema['enum']}", path)
    if "const" in schema and instance != schema["const"]:
        raise ValidationError(f"must equal {schema['const']!r}", path)
    if isinstance(instance, (int, float)) and not isinstance(instance, bool):
        if "minimum" in schema and instance < schema["minimum"]:
            raise ValidationError(f"{instance} < minimum {schema['minimum']}", path)
        if "maximum" in schema and instance > schema["maximum"]:
            raise ValidationError(f"{instance} > maximum {schema['maximum']}", path)
        if "exclusiveMinimum" in schema and instance <= schema["exclusiveMinimum"]:
            raise ValidationError(f"{instance} <= {schema['exclusiveMinimum']}", path)
    if isinstance(instance, str):
        if "minLength" in schema and len(instance) < schema["minLength"]:
            raise ValidationError("string too short", path)
        if "maxLength" in schema and len(instance) > schema["maxLength"]:
            raise ValidationError("string too long", path)
        if "pattern" in schema and not re.search(schema["pattern"], instance):
            raise ValidationError(f"does not match {schema['pattern']}", path)
    if isinstance(instance, dict):
        props = schema.get("properties", {})
        for r in schema.get("required", []):
            if r not in instance:
                raise ValidationError(f"missing required property '{r}'", path)
        pats = schema.get("patternProperties", {})
        addl = schema.get("additionalProperties", True)
        for k, v in instance.items():
            matched = False
            if k in props:
                validate(v, props[k], root, path + [k])
                matched = True
            for pat, sub in pats.items():
                if re.search(pat, k):
                    validate(v, sub, root, path + [k])
                    matched = True
            if not matched:
                if addl is False:
                    raise ValidationError(f"additional property '{k}' not allowed", path)
                if isinstance(addl, dict):
                    validate(v, addl, root, path + [k])
    if isinstance(instance, list):
        if "minItems" in schema and len(instance) < schema["minItems"]:
            raise ValidationError("too few items", path)
        if "maxItems" in schema and len(instance) > schema["maxItems"]:
            raise ValidationError("too many items", path)
        items = schema.get("items")
        if isinstance(items, dict):
            for i, v in enumerate(instance):
                validate(v, items, root, path + [i])
    if "allOf" in schema:
        for sub in schema["allOf"]:
            validate(instance, sub, root, path)
    if "anyOf" in schema:
        errs = []
        for sub in schema["anyOf"]:
            try:
                validate(instance, sub, root, path)
                break
            except ValidationError as e:
                errs.append(e)
        else:
            raise ValidationError("no anyOf branch matched: " + "; ".join(map(str, errs)), path)
    if "oneOf" in schema:
        ok = 0
        for sub in schema["oneOf"]:
            try:
                validate(instance, sub, root, path)
                ok += 1
            except ValidationError:
                pass
        if ok != 1:
            raise ValidationError(f"{ok} oneOf branches matched (need exactly 1)", path)
    if "not" in schema:
        try:
            validate(instance, schema["not"], root, path)
        except ValidationError:
            pass
        else:
            raise ValidationError("matched a 'not' schema", path)
