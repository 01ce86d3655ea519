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
               "hotspot_temp", "mem_temp", "gfx_clock", "mem_clock", "hbm_bw", "mfma_busy", "mfma_contention", "hbm_contention", "xgmi_read",
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


# ------------------------------------------------------------------------- JSON schemas
# OpenAPI 3.0 schema objects.  The SAME dicts are rendered into the document and enforced by
# :func:`validate` (request bodies at runtime; response bodies in tests/test_openapi_contract.py).
def _t(t: str, **kw) -> dict:
    return {"type": t, **kw}


STR, INT, BOOL, NUM = _t("string"), _t("integer"), _t("boolean"), _t("number")
DATE_TIME = _t("string", format="date-time", example="2026-01-01T10:00:00.000Z")
HOUR = _t("string", pattern=r"^([01]?\d|2[0-3]):[0-5]\d$", example="08:30")
WEEKDAYS = ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"]
JOB_STATUSES = ["not_running", "running", "terminated", "unsynchronized", "pending"]
TASK_STATUSES = ["not_running", "running", "terminated", "unsynchronized"]


def nullable(s: dict) -> dict:
    return {**s, "nullable": True}


def ref(name: str) -> dict:
    return {"$ref": f"#/components/schemas/{name}"}


def arr(item: dict, **kw) -> dict:
    return {"type": "array", "items": item, **kw}


def obj(props: dict, required=(), extra: bool = True, **kw) -> dict:
    d = {"type": "object", "properties": props, **kw}
    if required:
        d["required"] = list(required)
    if not extra:
        d["additionalProperties"] = False
    return d


def envelope(**fields) -> dict:
    """``{"msg": ..., <key>: <schema>}`` -- the controllers' usual success body."""
    return obj({"msg": STR, **fields}, required=["msg", *fields])


SCHEMAS: dict[str, dict] = {
    # --- request bodies
    "UserForm": obj({"username": _t("string", minLength=1, maxLength=40, example="foobar"),
                     "email": _t("string", example="foo@bar.com"),
                     "password": _t("string", example="difficult_password")},
                    required=["username", "email", "password"]),
    "UserUpdateForm": obj({"id": INT, "roles": arr(_t("string", enum=["user", "admin"])),
                           "username": _t("string", minLength=1, maxLength=40), "password": STR, "email": STR},
                          required=["id"]),
    "UserLoginForm": obj({"username": STR, "password": STR}, required=["username", "password"]),
    "PasswordChangeForm": obj({"oldPassword": STR, "newPassword": STR},  # new: self-service
                              required=["oldPassword", "newPassword"], extra=False),
    "CommandSegment": obj({"name": _t("string", minLength=1, maxLength=50), "value": STR}, required=["name"]),
    "CommandSegments": obj({"envs": arr(ref("CommandSegment")), "params": arr(ref("CommandSegment"))},
                           extra=False),
    "TaskForm": obj({"jobId": INT, "command": _t("string", maxLength=400), "hostname": _t("string", maxLength=40),
                     "cmdsegments": ref("CommandSegments"),
                     "maxRestarts": _t("integer", minimum=0, maximum=100)},  # new: restart policy
                    required=["command", "hostname"]),
    "TaskUpdateForm": obj({"command": _t("string", maxLength=400), "hostname": _t("string", maxLength=40),
                           "cmdsegments": ref("CommandSegments"),
                           "maxRestarts": _t("integer", minimum=0, maximum=100)}),
    # new: multi-task launch generator (torchrun / torch TCP ranks / TF2 TF_CONFIG / TF1 ClusterSpec)
    "TaskGenerateForm": obj({"template": STR, "command": STR, "module": STR,
                             "masterPort": _t("integer", minimum=1, maximum=65535),
                             "placements": arr(obj({"hostname": STR, "gpu": _t("integer", minimum=0),
                                                    "gpus": {"description": "[index, ...] or 'auto:N'"},
                                                    "gpuCount": _t("integer", minimum=1),
                                                    "role": _t("string", enum=["chief", "worker", "ps", "evaluator"])},
                                                   required=["hostname"]), minItems=1)},
                            required=["template", "placements"]),
    "JobForm": obj({"name": _t("string", minLength=1, maxLength=40), "description": STR, "userId": INT,
                    "startAt": nullable(DATE_TIME), "stopAt": nullable(DATE_TIME)}, required=["name", "userId"]),
    "JobUpdateForm": obj({"name": _t("string", minLength=1, maxLength=40), "description": STR,
                          "startAt": nullable(DATE_TIME), "stopAt": nullable(DATE_TIME)}),
    "GroupForm": obj({"name": _t("string", minLength=1, maxLength=40), "isDefault": BOOL}, required=["name"]),
    "GroupUpdateForm": obj({"name": _t("string", minLength=1, maxLength=40), "isDefault": BOOL}),
    "RestrictionForm": obj({"name": STR, "startsAt": DATE_TIME, "endsAt": nullable(DATE_TIME), "isGlobal": BOOL},
                           required=["startsAt", "isGlobal"]),
    "RestrictionUpdateForm": obj({"name": STR, "startsAt": DATE_TIME, "endsAt": nullable(DATE_TIME),
                                  "isGlobal": BOOL}),
    # day names and hours are checked by the controller: an unknown day is a 422 in TensorHive 1.1
    # (tests/functional/controllers/test_schedule_controller_superuser.py:51-59), not a 400
    "ScheduleForm": obj({"scheduleDays": arr(_t("string", example="Monday")), "hourStart": _t("string", example="8:00"),
                         "hourEnd": _t("string", example="16:00")}, required=["scheduleDays", "hourStart", "hourEnd"]),
    "ScheduleUpdateForm": obj({"scheduleDays": arr(_t("string", example="Monday")),
                               "hourStart": _t("string", example="8:00"), "hourEnd": _t("string", example="16:00")}),
    "ReservationForm": obj({"title": _t("string", maxLength=60), "description": _t("string", maxLength=200),
                            "resourceId": STR, "userId": INT, "start": DATE_TIME, "end": DATE_TIME},
                           required=["title", "description", "resourceId", "userId", "start", "end"]),
    "ReservationUpdateForm": obj({"title": _t("string", maxLength=60), "description": _t("string", maxLength=200),
                                  "resourceId": STR, "start": DATE_TIME, "end": DATE_TIME, "isCancelled": BOOL}),
    # --- display objects
    "GroupWithoutUsers": obj({"id": INT, "name": STR, "isDefault": BOOL, "createdAt": DATE_TIME},
                             required=["name", "isDefault"]),
    "UserWithoutGroup": obj({"id": INT, "username": STR, "createdAt": DATE_TIME, "roles": arr(STR),
                             "email": STR}),
    "UserToDisplay": obj({"id": INT, "username": STR, "createdAt": DATE_TIME, "roles": arr(STR), "email": STR,
                          "groups": arr(ref("GroupWithoutUsers"))}),
    "Group": obj({"id": INT, "name": STR, "isDefault": BOOL, "createdAt": DATE_TIME,
                  "users": arr(ref("UserWithoutGroup"))}, required=["name", "isDefault", "users"]),
    "Resource": obj({"id": STR, "name": nullable(STR), "hostname": nullable(STR)}),
    "Schedule": obj({"id": INT, "scheduleDays": arr(_t("string", enum=WEEKDAYS)), "hourStart": HOUR,
                     "hourEnd": HOUR}, required=["scheduleDays", "hourStart", "hourEnd"]),
    "Restriction": obj({"id": INT, "name": nullable(STR), "createdAt": DATE_TIME, "startsAt": DATE_TIME,
                        "endsAt": nullable(DATE_TIME), "isGlobal": BOOL, "schedules": arr(ref("Schedule")),
                        "groups": arr(ref("GroupWithoutUsers")), "users": arr(ref("UserWithoutGroup")),
                        "resources": arr(ref("Resource"))},
                       required=["name", "createdAt", "startsAt", "endsAt", "isGlobal", "schedules"]),
    "Reservation": obj({"id": INT, "title": STR, "description": STR, "resourceId": STR, "userId": INT,
                        "userName": nullable(STR), "start": DATE_TIME, "end": DATE_TIME, "createdAt": DATE_TIME,
                        "isCancelled": BOOL, "gpuUtilAvg": nullable(INT), "memUtilAvg": nullable(INT)},
                       required=["title", "description", "resourceId", "userId", "userName", "start", "end",
                                 "isCancelled", "gpuUtilAvg", "memUtilAvg"]),
    "JobToDisplay": obj({"id": INT, "name": STR, "description": nullable(STR), "userId": INT,
                         "status": _t("string", enum=JOB_STATUSES), "startAt": nullable(DATE_TIME),
                         "stopAt": nullable(DATE_TIME), "isQueued": nullable(BOOL),
                         "tasks": arr(ref("TaskToDisplay"))}),
    "CommandSegmentToDisplay": obj({"name": STR, "value": nullable(STR), "index": INT}),
    "TaskToDisplay": obj({"id": INT, "jobId": INT, "hostname": STR, "pid": nullable(INT), "command": STR,
                          "status": _t("string", enum=TASK_STATUSES),
                          "cmdsegments": obj({"envs": arr(ref("CommandSegmentToDisplay")),
                                              "params": arr(ref("CommandSegmentToDisplay"))}),
                          "fullCommand": STR, "gpuId": nullable(INT), "allocatedGpus": arr(INT),
                          "maxRestarts": INT, "restarts": INT}),
    "Metric": obj({"value": nullable(NUM), "unit": nullable(STR)}),
    "GPUProcess": obj({"pid": INT, "command": nullable(STR), "owner": nullable(STR), "task_id": nullable(STR),
                       "vram": nullable(NUM)}),
    "GPU": obj({"name": nullable(STR), "index": nullable(INT), "bdf": nullable(STR), "numa_node": nullable(INT),
                "metrics": obj({}, additionalProperties=ref("Metric")),
                "processes": nullable(arr(ref("GPUProcess")))}),
    "GPUAllData": obj({}, additionalProperties=obj({
        "GPU": nullable(obj({}, additionalProperties=ref("GPU"))),
        "CPU": nullable(obj({}, additionalProperties=obj({"name": STR, "index": INT,
                                                          "metrics": nullable(obj({}, additionalProperties=ref("Metric")))})))}),
        description="hostname -> {GPU: {uuid: GPU}, CPU: {CPU_<host>: {...}}}"),
    "GPUInfo": obj({}, additionalProperties=obj({"name": nullable(STR), "index": nullable(INT),
                                                 "bdf": nullable(STR), "numa_node": nullable(INT)}),
                   description="uuid -> static GPU facts"),
    "GPUMetricsInTwoCases": obj({}, additionalProperties=obj({}), description=(
        "uuid -> {metric: Metric} (all metrics) or uuid -> Metric (metric_type given)")),
    "CPUMetrics": obj({}, additionalProperties=obj({}), description="CPU_<host> -> {metric: Metric} or Metric"),
    "GPUProcesses": obj({}, additionalProperties=nullable(arr(ref("GPUProcess"))),
                        description="uuid -> processes on that GPU"),
    # --- generic bodies
    "Message": obj({"msg": STR}, required=["msg"]),
    "Problem": obj({"detail": STR, "status": INT, "title": STR, "type": STR}, required=["detail", "status"]),
    "TokenPair": obj({"msg": STR, "access_token": STR, "refresh_token": STR}, required=["access_token"]),
    # --- new operations
    "Topology": obj({}, additionalProperties=obj({}), description="hostname -> GPU link/NUMA topology"),
    "InternalMetrics": obj({}, description="services' loop statistics, request latency p50/p99, snapshot ages"),
    "Templates": obj({"templates": arr(obj({"name": STR}))}),
    "TrainingMetrics": obj({"msg": STR, "path": STR, "tokensPerSec": nullable(NUM),
                            "last": nullable(ref("TrainingPoint")), "series": arr(ref("TrainingPoint"))},
                           required=["series"]),
    "TrainingPoint": obj({"step": INT, "loss": NUM, "tokensPerSec": NUM, "world": nullable(INT)}),
}


# ------------------------------------------------------------------------- validation
class SchemaError(ValueError):
    pass


def _resolve_ref(s: dict) -> dict:
    while "$ref" in s:
        s = SCHEMAS[s["$ref"].rsplit("/", 1)[-1]]
    return s


_JSON_TYPES = {"string": (str,), "integer": (int,), "number": (int, float), "boolean": (bool,), "array": (list,),
               "object": (dict,)}


def _check_format(v: str, fmt: str, where: str) -> None:
    if fmt == "date-time":
        from ..utils.dates import parse

        try:
            parse(v)
        except (ValueError, TypeError):
            raise SchemaError(f"'{v}' is not a 'date-time' ({where})")


def validate(value, schema: dict, where: str = "body") -> None:
    """Validate ``value`` against an OpenAPI 3.0 schema object (subset: $ref, type, nullable, enum,
    format date-time, pattern, min/maxLength, minimum/maximum, items/minItems, properties,
    required, additionalProperties).  Raises :class:`SchemaError` naming the failing location."""
    import re

    s = _resolve_ref(schema)
    if value is None:
        if s.get("nullable"):
            return
        raise SchemaError(f"None is not of type '{s.get('type', 'object')}' ({where})")
    t = s.get("type")
    if t:
        ok = isinstance(value, _JSON_TYPES[t]) and not (t in ("integer", "number") and isinstance(value, bool))
        if not ok:
            raise SchemaError(f"{value!r} is not of type '{t}' ({where})")
    if "enum" in s and value not in s["enum"]:
        raise SchemaError(f"{value!r} is not one of {s['enum']} ({where})")
    if t == "string":
        if "minLength" in s and len(value) < s["minLength"]:
            raise SchemaError(f"{value!r} is too short ({where})")
        if "maxLength" in s and len(value) > s["maxLength"]:
            raise SchemaError(f"{value!r} is too long ({where})")
        if "pattern" in s and not re.search(s["pattern"], value):
            raise SchemaError(f"{value!r} does not match '{s['pattern']}' ({where})")
        if "format" in s:
            _check_format(value, s["format"], where)
    if t in ("integer", "number"):
        if "minimum" in s and value < s["minimum"]:
            raise SchemaError(f"{value!r} is less than the minimum of {s['minimum']} ({where})")
        if "maximum" in s and value > s["maximum"]:
            raise SchemaError(f"{value!r} is greater than the maximum of {s['maximum']} ({where})")
    if t == "array":
        if "minItems" in s and len(value) < s["minItems"]:
            raise SchemaError(f"{value!r} has fewer than {s['minItems']} items ({where})")
        for i, v in enumerate(value):
            validate(v, s.get("items", {}), f"{where}[{i}]")
    if t == "object" or "properties" in s:
        for f in s.get("required", []):
            if f not in value:
                raise SchemaError(f"'{f}' is a required property ({where})")
        props = s.get("properties", {})
        extra = s.get("additionalProperties", True)
        for k, v in value.items():
            if k in props:
                validate(v, props[k], f"{where}.{k}")
            elif extra is False:
                raise SchemaError(f"Additional property '{k}' is not allowed ({where})")
            elif isinstance(extra, dict):
                validate(v, extra, f"{where}.{k}")


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
    Op("GET", "/metrics/prometheus", "nodes.get_prometheus", "scrape", tag="nodes"),                  # new
    Op("POST", "/jobs/{id}/tasks/generate", "job.generate_tasks", "jwt", [P("id")],              # new
       body="TaskGenerateForm", body_name="form", tag="jobs"),
    Op("PUT", "/jobs/{id}/reservation/{reservation_id}", "job.attach_to_reservation", "jwt",      # new
       [P("id"), P("reservation_id"), Q("siblings", "boolean")], tag="jobs"),
    Op("PUT", "/user/password", "user.change_password", "jwt", body="PasswordChangeForm",         # new
       body_name="form", tag="users"),
    Op("GET", "/tasks/{id}/training", "task.get_training_metrics", "jwt",                       # new
       ID + [Q("lines", "integer")], tag="tasks"),
]

COMPAT_OPERATION_COUNT = 66
assert len(OPERATIONS) == COMPAT_OPERATION_COUNT, len(OPERATIONS)


# ------------------------------------------------------------------------- responses
# handler -> (success status, success body schema, error statuses).  Status sets are a superset
# of the reference document's (tests/fixtures/reference_openapi_contract.json).
def _env(key: str, schema_name: str) -> dict:
    return envelope(**{key: ref(schema_name)})


def _env_list(key: str, schema_name: str) -> dict:
    return envelope(**{key: arr(ref(schema_name))})


_R = ref("Restriction")
RESPONSES: dict[str, tuple[int, dict | None, tuple[int, ...]]] = {
    "user.get": (200, arr(ref("UserToDisplay")), (401, 403, 422)),
    "user.get_by_id": (200, _env("user", "UserToDisplay"), (401, 403, 404, 422, 500)),
    "user.create": (201, _env("user", "UserToDisplay"), (400, 401, 403, 409, 422, 500)),
    "user.update": (201, _env("user", "UserToDisplay"), (400, 401, 403, 404, 409, 422, 500)),
    "user.ssh_signup": (201, _env("user", "UserToDisplay"), (400, 403, 409, 422, 500)),
    "user.delete": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "user.logout_with_access_token": (200, ref("Message"), (401, 422, 500)),
    "user.logout_with_refresh_token": (200, ref("Message"), (401, 422, 500)),
    "user.generate": (200, obj({"access_token": STR}, required=["access_token"]), (401, 422)),
    "user.login": (200, ref("TokenPair"), (400, 401, 404, 422, 500)),
    "user.authorized_keys_entry": (200, obj({}), (500,)),
    "user.change_password": (200, ref("Message"), (400, 401, 403, 422)),
    "group.get": (200, arr(ref("Group")), (400, 401, 403, 422)),
    "group.create": (201, _env("group", "Group"), (400, 401, 403, 422, 500)),
    "group.get_by_id": (200, _env("group", "Group"), (401, 404, 422, 500)),
    "group.update": (200, _env("group", "Group"), (400, 401, 403, 404, 422, 500)),
    "group.delete": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "group.add_user": (200, _env("group", "Group"), (401, 403, 404, 409, 422, 500)),
    "group.remove_user": (200, _env("group", "Group"), (401, 403, 404, 422, 500)),
    "restriction.get": (200, arr(_R), (400, 401, 403, 422, 500)),
    "restriction.create": (201, _env("restriction", "Restriction"), (400, 401, 403, 422, 500)),
    "restriction.update": (200, _env("restriction", "Restriction"), (400, 401, 403, 404, 422, 500)),
    "restriction.delete": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "schedule.get": (200, arr(ref("Schedule")), (401, 403, 422, 500)),
    "schedule.create": (201, _env("schedule", "Schedule"), (400, 401, 403, 422, 500)),
    "schedule.get_by_id": (200, _env("schedule", "Schedule"), (401, 404, 422, 500)),
    "schedule.update": (200, _env("schedule", "Schedule"), (400, 401, 403, 404, 422, 500)),
    "schedule.delete": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "job.get_all": (200, _env_list("jobs", "JobToDisplay"), (400, 401, 403, 422, 500)),
    "job.create": (201, _env("job", "JobToDisplay"), (400, 401, 403, 409, 422, 500)),
    "job.get_by_id": (200, _env("job", "JobToDisplay"), (401, 403, 404, 422, 500)),
    "job.update": (200, _env("job", "JobToDisplay"), (400, 401, 403, 404, 422, 500)),
    "job.delete": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "job.execute": (200, _env("job", "JobToDisplay"), (401, 403, 404, 409, 422, 500)),
    "job.enqueue": (200, _env("job", "JobToDisplay"), (401, 403, 404, 409, 422, 500)),
    "job.dequeue": (200, _env("job", "JobToDisplay"), (401, 403, 404, 409, 422, 500)),
    "job.stop": (200, _env("job", "JobToDisplay"), (401, 403, 404, 409, 422, 500)),
    "job.add_task": (200, _env("job", "JobToDisplay"), (401, 403, 404, 409, 422, 500)),
    "job.remove_task": (200, _env("job", "JobToDisplay"), (401, 403, 404, 422, 500)),
    "task.create": (201, _env("task", "TaskToDisplay"), (400, 401, 403, 404, 409, 422, 500)),
    "reservation.get": (200, arr(ref("Reservation")), (400, 401, 422, 500)),
    "reservation.create": (201, _env("reservation", "Reservation"), (400, 401, 403, 422, 500)),
    "reservation.update": (201, _env("reservation", "Reservation"), (400, 401, 403, 404, 422, 500)),
    "reservation.delete": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "resource.get": (200, arr(ref("Resource")), (401, 403, 422)),
    "resource.get_by_id": (200, _env("resource", "Resource"), (401, 404, 422, 500)),
    "nodes.get_hostnames": (200, arr(STR), (401, 422)),
    "nodes.get_all_data": (200, ref("GPUAllData"), (401, 422)),
    "nodes.get_gpu_info": (200, ref("GPUInfo"), (401, 404, 422)),
    "nodes.get_gpu_metrics": (200, ref("GPUMetricsInTwoCases"), (400, 401, 404, 422)),
    "nodes.get_cpu_metrics": (200, ref("CPUMetrics"), (400, 401, 404, 422)),
    "nodes.get_gpu_processes": (200, ref("GPUProcesses"), (401, 404, 422)),
    "task.get_all": (200, _env_list("tasks", "TaskToDisplay"), (400, 401, 403, 404, 422, 500)),
    "task.get": (200, _env("task", "TaskToDisplay"), (401, 403, 404, 422, 500)),
    "task.update": (201, _env("task", "TaskToDisplay"), (400, 401, 403, 404, 422, 500)),
    "task.destroy": (200, ref("Message"), (401, 403, 404, 422, 500)),
    "task.get_log": (200, envelope(path=STR, output_lines=arr(STR)), (401, 403, 404, 422, 500)),
    # new operations
    "nodes.get_topology": (200, ref("Topology"), (401, 422)),
    "nodes.get_internal_metrics": (200, ref("InternalMetrics"), (401, 403, 422)),
    "nodes.get_prometheus": (200, None, (401, 403, 422)),
    "job.get_templates": (200, obj({"msg": STR, "templates": obj({}, additionalProperties=obj({}))}), (401, 422)),
    "job.generate_tasks": (201, _env_list("tasks", "TaskToDisplay"), (400, 401, 403, 404, 422, 500)),
    "job.attach_to_reservation": (200, _env("job", "JobToDisplay"), (400, 401, 403, 404, 409, 422, 500)),
    "task.get_training_metrics": (200, ref("TrainingMetrics"), (401, 403, 404, 422, 500)),
}
for _h in ("apply_to_user", "remove_from_user", "apply_to_group", "remove_from_group", "apply_to_resource",
           "remove_from_resource", "apply_to_resources_by_hostname", "remove_from_resources_by_hostname",
           "add_schedule", "remove_schedule"):
    RESPONSES[f"restriction.{_h}"] = (200, _env("restriction", "Restriction"), (400, 401, 403, 404, 409, 422, 500))

_ERROR_TEXT = {400: ("general", "bad_request"), 401: ("general", "unauthorized"), 403: ("general", "unprivileged"),
               404: None, 409: None, 422: ("general", "auth_error"), 500: ("general", "internal_error")}
_ERROR_FALLBACK = {404: "Not found", 409: "Conflict with the current state"}


def _message(responses: dict | None, keys) -> str | None:
    cur = responses or {}
    for k in keys:
        if not isinstance(cur, dict) or k not in cur:
            return None
        cur = cur[k]
    return cur if isinstance(cur, str) else None


def _op_responses(op: Op, messages: dict | None) -> dict:
    ok, body, errors = RESPONSES[op.handler]
    entity = op.handler.split(".", 1)[0]
    out: dict = {}
    desc = _message(messages, (entity, op.handler.split(".", 1)[1], "success")) or \
        _message(messages, ("general", "success")) or "OK"
    out[str(ok)] = {"description": desc}
    if body is not None:
        out[str(ok)]["content"] = {"application/json": {"schema": body}}
    elif op.handler == "nodes.get_prometheus":
        out[str(ok)]["content"] = {"text/plain": {"schema": STR}}
    for code in errors:
        if code == 404:
            d = _message(messages, (entity, "not_found"))
        else:
            keys = _ERROR_TEXT.get(code)
            d = _message(messages, keys) if keys else None
        d = d or _ERROR_FALLBACK.get(code, "Error")
        sch = ref("Problem") if code == 400 else ref("Message")
        out[str(code)] = {"description": d, "content": {"application/json": {"schema": sch}}}
    return out


def openapi_document(title: str, prefix: str, version: str, messages: dict | None = None) -> dict:
    """Render the OpenAPI 3.0.3 document for every operation: parameters, request bodies, every
    response status with its body schema, and the component schemas they reference."""
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
                       "summary": op.summary or op.handler.replace(".", " ").replace("_", " "),
                       "parameters": params, "responses": _op_responses(op, messages)}
        if op.auth is None:
            entry["security"] = []
        else:
            entry["security"] = [{"Bearer": []}]
            entry["x-auth"] = op.auth
        if op.body:
            entry["requestBody"] = {"required": True, "x-body-name": op.body_name,
                                    "content": {"application/json": {"schema": ref(op.body)}}}
        item[op.method.lower()] = entry
    return {
        "openapi": "3.0.3",
        "info": {"title": title, "version": version},
        "servers": [{"url": f"/{prefix}"}],
        "paths": paths,
        "components": {"schemas": SCHEMAS,
                       "parameters": {
                           "gpuMetricTypeQuery": {"name": "metric_type", "in": "query", "required": False,
                                                  "schema": {"type": "string", "enum": GPU_METRICS}},
                           "cpuMetricTypeQuery": {"name": "metric_type", "in": "query", "required": False,
                                                  "schema": {"type": "string", "enum": CPU_METRICS}}},
                       "securitySchemes": {"Bearer": {"type": "http", "scheme": "bearer", "bearerFormat": "JWT"}}},
    }
