"""Declarative REST surface: 66 operations + request schemas -> router table AND OpenAPI 3 doc.

The reference drives connexion from a 3.8k-line hand-written YAML spec
(``api/api_specification.yml``).  Here the single source of truth is this Python table; the
OpenAPI 3.0.3 document served at ``/{prefix}/openapi.json`` is generated from it, and the same
table drives the strict request validator in :mod:`.app`.  Paths, parameter names, body field
names, auth requirements and status codes are those of TensorHive 1.1;
additions are marked ``# new``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

GPU_METRICS = ["fan_speed", "mem_free", "mem_used", "mem_total", "utilization", "mem_util", "temp", "power",
               # new (MI355X telemetry)
               "hotspot_temp", "mem_temp", "gfx_clock", "mem_clock", "hbm_bw", "mfma_busy", "hbm_contention", "xgmi_read",
               "xgmi_write", "energy"]
CPU_METRICS = ["mem_free", "mem_used", "mem_total", "utilization"]


@dataclass
class Param:
    name: str
    where: str  # "path" | "query"
    type: str  # integer | string | boolean | number | array
    required: bool = False
    nullable: bool = False
    enum: list | None = None
    items: str = "string"


@dataclass
class Op:
    method: str
    path: str
    handler: str  # "module.function" under tensorhive_fixed_amd.controllers
    auth: str | None  # None | "jwt" | "admin" | "refresh"
    params: list[Param] = field(default_factory=list)
    body: str | None = None  # schema name
    body_name: str | None = None  # kwarg the body is passed as (x-body-name)
    summary: str = ""
    tag: str = ""


def P(name, t="integer", where="path", **kw):
    return Param(name, where, t, required=(where == "path") or kw.pop("required", False), **kw)


def Q(name, t="string", **kw):
    return Param(name, "query", t, **kw)


# ---- request body schemas: {field: (type, nullable)} + required
SCHEMAS: dict[str, dict] = {
    "UserForm": {"required": ["username", "email", "password"],
                 "properties": {"username": "string", "email": "string", "password": "string"}},
    "UserUpdateForm": {"required": ["id"],
                       "properties": {"id": "integer", "roles": "array", "username": "string", "password": "string",
                                      "email": "string"}},
    "UserLoginForm": {"required": ["username", "password"],
                      "properties": {"username": "string", "password": "string"}},
    "TaskForm": {"required": ["command", "hostname"],
                 "properties": {"jobId": "integer", "command": "string", "hostname": "string", "cmdsegments": "object",
                                "maxRestarts": "integer"}},
    "TaskUpdateForm": {"required": [], "properties": {"command": "string", "hostname": "string", "cmdsegments": "object",
                                                    "maxRestarts": "integer"}},
    # new: multi-task launch generator (torchrun / torch TCP ranks / TF2 TF_CONFIG / TF1 ClusterSpec)
    "TaskGenerateForm": {"required": ["template", "placements"],
                         "properties": {"template": "string", "command": "string", "module": "string",
                                        "placements": "array", "masterPort": "integer"}},
    "JobForm": {"required": ["name", "userId"],
                "properties": {"name": "string", "description": "string", "userId": "integer", "startAt": "string?",
                               "stopAt": "string?"}},
    "JobUpdateForm": {"required": [], "properties": {"name": "string", "description": "string", "startAt": "string?",
                                                     "stopAt": "string?"}},
    "GroupForm": {"required": ["name"], "properties": {"name": "string", "isDefault": "boolean"}},
    "GroupUpdateForm": {"required": [], "properties": {"name": "string", "isDefault": "boolean"}},
    "RestrictionForm": {"required": ["startsAt", "isGlobal"],
                        "properties": {"name": "string", "startsAt": "string", "endsAt": "string?", "isGlobal": "boolean"}},
    "RestrictionUpdateForm": {"required": [], "properties": {"name": "string", "startsAt": "string", "endsAt": "string?",
                                                             "isGlobal": "boolean"}},
    "ScheduleForm": {"required": ["scheduleDays", "hourStart", "hourEnd"],
                     "properties": {"scheduleDays": "array", "hourStart": "string", "hourEnd": "string"}},
    "ScheduleUpdateForm": {"required": [], "properties": {"scheduleDays": "array", "hourStart": "string",
                                                          "hourEnd": "string"}},
    "ReservationForm": {"required": ["title", "description", "resourceId", "userId", "start", "end"],
                        "properties": {"title": "string", "description": "string", "resourceId": "string",
                                       "userId": "integer", "start": "string", "end": "string"}},
    "ReservationUpdateForm": {"required": [], "properties": {"title": "string", "description": "string",
                                                             "resourceId": "string", "start": "string", "end": "string",
                                                             "isCancelled": "boolean"}},
}

ID = [P("id")]

OPERATIONS: list[Op] = [
    # users / auth
    Op("GET", "/users", "user.get", "jwt", tag="users"),
    Op("GET", "/users/{id}", "user.get_by_id", "jwt", ID, tag="users"),
    Op("POST", "/user/create", "user.create", "admin", body="UserForm", body_name="newUser", tag="users"),
    Op("PUT", "/user", "user.update", "admin", body="UserUpdateForm", body_name="newValues", tag="users"),
    Op("POST", "/user/ssh_signup", "user.ssh_signup", None, body="UserForm", body_name="user", tag="users"),
    Op("DELETE", "/user/delete/{id}", "user.delete", "admin", ID, tag="users"),
    Op("DELETE", "/user/logout", "user.logout_with_access_token", "jwt", tag="auth"),
    Op("DELETE", "/user/logout/refresh_token", "user.logout_with_refresh_token", "refresh", tag="auth"),
    Op("GET", "/user/refresh", "user.generate", "refresh", tag="auth"),
    Op("POST", "/user/login", "user.login", None, body="UserLoginForm", body_name="user", tag="auth"),
    Op("GET", "/user/authorized_keys_entry", "user.authorized_keys_entry", None, tag="auth"),
    # groups
    Op("GET", "/groups", "group.get", "jwt", [Q("only_default", "boolean")], tag="groups"),
    Op("POST", "/groups", "group.create", "admin", body="GroupForm", body_name="group", tag="groups"),
    Op("GET", "/groups/{id}", "group.get_by_id", "jwt", ID, tag="groups"),
    Op("PUT", "/groups/{id}", "group.update", "admin", ID, body="GroupUpdateForm", body_name="newValues", tag="groups"),
    Op("DELETE", "/groups/{id}", "group.delete", "admin", ID, tag="groups"),
    Op("PUT", "/groups/{group_id}/users/{user_id}", "group.add_user", "admin", [P("group_id"), P("user_id")], tag="groups"),
    Op("DELETE", "/groups/{group_id}/users/{user_id}", "group.remove_user", "admin", [P("group_id"), P("user_id")],
       tag="groups"),
    # restrictions
    Op("GET", "/restrictions", "restriction.get", "jwt",
       [Q("user_id", "integer", nullable=True), Q("include_user_groups", "boolean", nullable=True),
        Q("group_id", "integer", nullable=True), Q("resource_id", "string", nullable=True),
        Q("schedule_id", "integer", nullable=True)], tag="restrictions"),
    Op("POST", "/restrictions", "restriction.create", "admin", body="RestrictionForm", body_name="restriction",
       tag="restrictions"),
    Op("PUT", "/restrictions/{id}", "restriction.update", "admin", ID, body="RestrictionUpdateForm",
       body_name="newValues", tag="restrictions"),
    Op("DELETE", "/restrictions/{id}", "restriction.delete", "admin", ID, tag="restrictions"),
    Op("PUT", "/restrictions/{restriction_id}/users/{user_id}", "restriction.apply_to_user", "admin",
       [P("restriction_id"), P("user_id")], tag="restrictions"),
    Op("DELETE", "/restrictions/{restriction_id}/users/{user_id}", "restriction.remove_from_user", "admin",
       [P("restriction_id"), P("user_id")], tag="restrictions"),
    Op("PUT", "/restrictions/{restriction_id}/groups/{group_id}", "restriction.apply_to_group", "admin",
       [P("restriction_id"), P("group_id")], tag="restrictions"),
    Op("DELETE", "/restrictions/{restriction_id}/groups/{group_id}", "restriction.remove_from_group", "admin",
       [P("restriction_id"), P("group_id")], tag="restrictions"),
    Op("PUT", "/restrictions/{restriction_id}/resources/{resource_uuid}", "restriction.apply_to_resource", "admin",
       [P("restriction_id"), P("resource_uuid", "string")], tag="restrictions"),
    Op("DELETE", "/restrictions/{restriction_id}/resources/{resource_uuid}", "restriction.remove_from_resource",
       "admin", [P("restriction_id"), P("resource_uuid", "string")], tag="restrictions"),
    Op("PUT", "/restrictions/{restriction_id}/hosts/{hostname}", "restriction.apply_to_resources_by_hostname",
       "admin", [P("restriction_id"), P("hostname", "string")], tag="restrictions"),
    Op("DELETE", "/restrictions/{restriction_id}/hosts/{hostname}",
       "restriction.remove_from_resources_by_hostname", "admin", [P("restriction_id"), P("hostname", "string")],
       tag="restrictions"),
    Op("PUT", "/restrictions/{restriction_id}/schedules/{schedule_id}", "restriction.add_schedule", "admin",
       [P("restriction_id"), P("schedule_id")], tag="restrictions"),
    Op("DELETE", "/restrictions/{restriction_id}/schedules/{schedule_id}", "restriction.remove_schedule", "admin",
       [P("restriction_id"), P("schedule_id")], tag="restrictions"),
    # schedules
    Op("GET", "/schedules", "schedule.get", "jwt", tag="schedules"),
    Op("POST", "/schedules", "schedule.create", "admin", body="ScheduleForm", body_name="schedule", tag="schedules"),
    Op("GET", "/schedules/{id}", "schedule.get_by_id", "jwt", ID, tag="schedules"),
    Op("PUT", "/schedules/{id}", "schedule.update", "admin", ID, body="ScheduleUpdateForm", body_name="newValues",
       tag="schedules"),
    Op("DELETE", "/schedules/{id}", "schedule.delete", "admin", ID, tag="schedules"),
    # jobs
    Op("GET", "/jobs", "job.get_all", "jwt", [Q("userId", "integer", nullable=True)], tag="jobs"),
    Op("POST", "/jobs", "job.create", "jwt", body="JobForm", body_name="job", tag="jobs"),
    Op("GET", "/jobs/{id}", "job.get_by_id", "jwt", ID, tag="jobs"),
    Op("PUT", "/jobs/{id}", "job.update", "jwt", ID, body="JobUpdateForm", body_name="newValues", tag="jobs"),
    Op("DELETE", "/jobs/{id}", "job.delete", "jwt", ID, tag="jobs"),
    Op("GET", "/jobs/{id}/execute", "job.execute", "jwt", ID, tag="jobs"),
    Op("PUT", "/jobs/{id}/enqueue", "job.enqueue", "jwt", ID, tag="jobs"),
    Op("PUT", "/jobs/{id}/dequeue", "job.dequeue", "jwt", ID, tag="jobs"),
    Op("GET", "/jobs/{id}/stop", "job.stop", "jwt", ID + [Q("gracefully", "boolean", nullable=True)], tag="jobs"),
    Op("POST", "/jobs/{job_id}/tasks", "task.create", "jwt", [P("job_id")], body="TaskForm", body_name="task",
       tag="jobs"),
    Op("PUT", "/jobs/{job_id}/tasks/{task_id}", "job.add_task", "jwt", [P("job_id"), P("task_id")], tag="jobs"),
    Op("DELETE", "/jobs/{job_id}/tasks/{task_id}", "job.remove_task", "jwt", [P("job_id"), P("task_id")], tag="jobs"),
    # reservations / resources
    Op("GET", "/reservations", "reservation.get", "jwt",
       [Q("resources_ids", "array"), Q("start", "string"), Q("end", "string")], tag="reservations"),
    Op("POST", "/reservations", "reservation.create", "jwt", body="ReservationForm", body_name="reservation",
       tag="reservations"),
    Op("PUT", "/reservations/{id}", "reservation.update", "jwt", ID, body="ReservationUpdateForm",
       body_name="newValues", tag="reservations"),
    Op("DELETE", "/reservations/{id}", "reservation.delete", "jwt", ID, tag="reservations"),
    Op("GET", "/resources", "resource.get", "jwt", tag="resources"),
    Op("GET", "/resource/{uuid}", "resource.get_by_id", "jwt", [P("uuid", "string")], tag="resources"),
    # nodes (monitoring)
    Op("GET", "/nodes/hostnames", "nodes.get_hostnames", "jwt", tag="nodes"),
    Op("GET", "/nodes/metrics", "nodes.get_all_data", "jwt", tag="nodes"),
    Op("GET", "/nodes/{hostname}/gpu/info", "nodes.get_gpu_info", "jwt", [P("hostname", "string")], tag="nodes"),
    Op("GET", "/nodes/{hostname}/gpu/metrics", "nodes.get_gpu_metrics", "jwt",
       [P("hostname", "string"), Q("metric_type", "string", enum=GPU_METRICS)], tag="nodes"),
    Op("GET", "/nodes/{hostname}/cpu/metrics", "nodes.get_cpu_metrics", "jwt",
       [P("hostname", "string"), Q("metric_type", "string", enum=CPU_METRICS)], tag="nodes"),
    Op("GET", "/nodes/{hostname}/gpu/processes", "nodes.get_gpu_processes", "jwt", [P("hostname", "string")],
       tag="nodes"),
    # tasks
    Op("GET", "/tasks", "task.get_all", "jwt", [Q("jobId", "integer", nullable=True), Q("syncAll", "boolean")],
       tag="tasks"),
    Op("GET", "/tasks/{id}", "task.get", "jwt", ID, tag="tasks"),
    Op("PUT", "/tasks/{id}", "task.update", "jwt", ID, body="TaskUpdateForm", body_name="newValues", tag="tasks"),
    Op("DELETE", "/tasks/{id}", "task.destroy", "jwt", ID, tag="tasks"),
    Op("GET", "/tasks/{id}/log", "task.get_log", "jwt", ID + [Q("tail", "boolean")], tag="tasks"),
]

# new, additive operations (not part of the 66 compat operations)
EXTRA_OPERATIONS: list[Op] = [
    Op("GET", "/nodes/topology", "nodes.get_topology", "jwt", tag="nodes"),                       # new
    Op("GET", "/metrics/internal", "nodes.get_internal_metrics", "admin", tag="nodes"),            # new
    Op("GET", "/jobs/templates", "job.get_templates", "jwt", tag="jobs"),                         # new
    Op("GET", "/metrics/prometheus", "nodes.get_prometheus", None, tag="nodes"),                  # new
    Op("POST", "/jobs/{id}/tasks/generate", "job.generate_tasks", "jwt", [P("id")],              # new
       body="TaskGenerateForm", body_name="form", tag="jobs"),
    Op("PUT", "/jobs/{id}/reservation/{reservation_id}", "job.attach_to_reservation", "jwt",      # new
       [P("id"), P("reservation_id"), Q("siblings", "boolean")], tag="jobs"),
    Op("GET", "/tasks/{id}/training", "task.get_training_metrics", "jwt",                       # new
       ID + [Q("lines", "integer")], tag="tasks"),
]

COMPAT_OPERATION_COUNT = 66
assert len(OPERATIONS) == COMPAT_OPERATION_COUNT, len(OPERATIONS)


def _oa_type(t: str) -> dict:
    nullable = t.endswith("?")
    t = t.rstrip("?")
    d: dict = {"type": t}
    if t == "array":
        d["items"] = {"type": "string"}
    if nullable:
        d["nullable"] = True
    return d


def openapi_document(title: str, prefix: str, version: str) -> dict:
    """Render the OpenAPI 3.0.3 document for every operation."""
    paths: dict = {}
    for op in OPERATIONS + EXTRA_OPERATIONS:
        item = paths.setdefault(op.path, {})
        params = []
        for p in op.params:
            sch: dict = {"type": p.type}
            if p.enum:
                sch["enum"] = list(p.enum)
            if p.nullable:
                sch["nullable"] = True
            if p.type == "array":
                sch["items"] = {"type": p.items}
            params.append({"name": p.name, "in": p.where, "required": p.required, "schema": sch})
        entry: dict = {"operationId": f"tensorhive_fixed_amd.controllers.{op.handler}", "tags": [op.tag],
                       "parameters": params, "responses": {"200": {"description": "OK"}}}
        if op.auth is None:
            entry["security"] = []
        if op.body:
            entry["requestBody"] = {"required": True, "x-body-name": op.body_name,
                                    "content": {"application/json": {"schema": {"$ref": f"#/components/schemas/{op.body}"}}}}
        item[op.method.lower()] = entry
    schemas = {}
    for name, s in SCHEMAS.items():
        sch = {"type": "object", "properties": {k: _oa_type(v) for k, v in s["properties"].items()}}
        if s["required"]:
            sch["required"] = list(s["required"])
        schemas[name] = sch
    return {
        "openapi": "3.0.3",
        "info": {"title": title, "version": version},
        "servers": [{"url": f"/{prefix}"}],
        "paths": paths,
        "components": {"schemas": schemas,
                       "securitySchemes": {"Bearer": {"type": "http", "scheme": "bearer", "bearerFormat": "JWT"}}},
        "security": [{"Bearer": []}],
    }
