"""GPU resources (reference ``controllers/resource.py``); both reads register new GPUs first."""
from __future__ import annotations

from ..models.orm import Resource
from ._common import M, guarded
from .nodes import register_resources_from_snapshot


def get():
    register_resources_from_snapshot()
    return [r.as_dict() for r in Resource.all()], 200


@guarded(not_found="resource.not_found")
def get_by_id(uuid: str):
    register_resources_from_snapshot()
    return {"msg": M("resource.get.success"), "resource": Resource.get(uuid).as_dict()}, 200
