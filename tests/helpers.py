"""Test helpers shared by API tests."""
import json


def api(client, method, path, headers=None, body=None, **q):
    headers = dict(headers or {})
    if body is not None:
        headers.setdefault("Content-Type", "application/json")
    resp = getattr(client, method)("/api" + path, headers=headers, data=None if body is None else json.dumps(body),
                                   query_string=q or None)
    try:
        data = resp.get_json()
    except Exception:  # noqa: BLE001
        data = None
    return resp.status_code, data
