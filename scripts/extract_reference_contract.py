#!/usr/bin/env python3
"""One-off: reduce the reference's OpenAPI document (``tensorhive/api/api_specification.yml``, a
Jinja-templated YAML) to its CONTRACT -- paths, methods, parameter names/locations/required,
request-body schema names, response status codes, component schema property names, required
sets and enums -- and write it as a committed JSON fixture (``tests/fixtures/
reference_openapi_contract.json``).  ``tests/test_openapi_contract.py`` checks our generated
document against that fixture, so the tests never need the reference tree.

``{{ ... }}`` template expressions are replaced by a placeholder string before parsing
(``yaml.safe_load``: nothing in the file is executed)."""
import json
import re
import sys
from pathlib import Path

import yaml

SRC = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tensorhive/api/api_specification.yml")
DST = Path(__file__).resolve().parents[1] / "tests" / "fixtures" / "reference_openapi_contract.json"


def _ref_name(schema):
    if not isinstance(schema, dict):
        return None
    if "$ref" in schema:
        return schema["$ref"].rsplit("/", 1)[-1]
    if schema.get("type") == "array" and isinstance(schema.get("items"), dict) and "$ref" in schema["items"]:
        return "array:" + schema["items"]["$ref"].rsplit("/", 1)[-1]
    return None


def _collect_enums(node, path, out):
    if isinstance(node, dict):
        if "enum" in node and isinstance(node["enum"], list):
            out[path] = [str(v) for v in node["enum"]]
        for k, v in node.items():
            _collect_enums(v, f"{path}.{k}" if path else str(k), out)
    elif isinstance(node, list):
        for i, v in enumerate(node):
            _collect_enums(v, f"{path}[{i}]", out)


def main():
    text = re.sub(r"\{\{.*?\}\}", "PLACEHOLDER", SRC.read_text())
    doc = yaml.safe_load(text)
    comps = doc.get("components", {})
    shared_params = comps.get("parameters", {})
    ops = []
    for path, item in doc["paths"].items():
        for method, op in item.items():
            if method not in ("get", "put", "post", "delete", "patch"):
                continue
            params = []
            for p in op.get("parameters", []) or []:
                if "$ref" in p:
                    p = shared_params[p["$ref"].rsplit("/", 1)[-1]]
                sch = p.get("schema", {}) or {}
                params.append({"name": p["name"], "in": p["in"], "required": bool(p.get("required", False)),
                               "type": sch.get("type"), "enum": [str(e) for e in sch.get("enum", [])] or None})
            body = None
            rb = op.get("requestBody")
            if rb:
                sch = (rb.get("content", {}).get("application/json", {}) or {}).get("schema", {})
                body = {"schema": _ref_name(sch), "x-body-name": rb.get("x-body-name"),
                        "required": bool(rb.get("required", False))}
            responses = {}
            for code, r in (op.get("responses") or {}).items():
                sch = (((r or {}).get("content") or {}).get("application/json") or {}).get("schema") or {}
                props = sorted((sch.get("properties") or {}).keys()) if isinstance(sch, dict) else []
                refs = {k: _ref_name(v) for k, v in (sch.get("properties") or {}).items()} if isinstance(sch, dict) else {}
                responses[str(code)] = {"schema": _ref_name(sch), "properties": props,
                                        "refs": {k: v for k, v in refs.items() if v}}
            ops.append({"path": path, "method": method, "operationId": op.get("operationId"),
                        "security": op.get("security"), "parameters": params, "requestBody": body,
                        "responses": responses})
    schemas = {}
    for name, s in (comps.get("schemas") or {}).items():
        schemas[name] = {"type": s.get("type"), "required": sorted(s.get("required", []) or []),
                         "properties": {k: {"type": (v or {}).get("type"), "ref": _ref_name(v)}
                                        for k, v in (s.get("properties") or {}).items()}}
    enums = {}
    _collect_enums(doc, "", enums)
    out = {"source": "tensorhive/api/api_specification.yml (TensorHive 1.1.0)", "openapi": doc.get("openapi"),
           "operations": ops, "schemas": schemas, "enums": enums,
           "securitySchemes": sorted((comps.get("securitySchemes") or {}).keys())}
    DST.parent.mkdir(parents=True, exist_ok=True)
    DST.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(f"{len(ops)} operations, {len(schemas)} schemas, {len(enums)} enums -> {DST}")


if __name__ == "__main__":
    main()
