"""Controller tests through the real HTTP router, for both roles (reference
``tests/functional/controllers/*`` -- there they patch the JWT decorators and call the view
functions; here every request carries a real token and passes spec validation)."""
import datetime
from datetime import timedelta

import pytest

from tensorhive_fixed_amd.models.orm import (Group, Job, Reservation, Resource, Restriction, RestrictionSchedule,
                                             Task, User)
from tensorhive_fixed_amd.database import db_session
from tests.helpers import api

UTC = datetime.datetime.utcnow
FMT = "%Y-%m-%dT%H:%M:%S.%fZ"


def iso(d):
    return d.strftime(FMT)


@pytest.fixture()
def as_user(client, new_user, auth_headers):
    h = auth_headers(new_user)
    return lambda method, path, body=None, **q: api(client, method, path, h, body, **q)


@pytest.fixture()
def as_admin(client, new_admin, auth_headers):
    h = auth_headers(new_admin)
    return lambda method, path, body=None, **q: api(client, method, path, h, body, **q)


# ============================================================================ users
def test_signup_requires_admin(as_user):
    st, _ = as_user("post", "/user/create", {"username": "someone", "email": "a@b.org", "password": "password1"})
    assert st == 403


def test_signup_joins_default_groups(as_admin, tables):
    g1 = Group(name="defaults1", is_default=True)
    g1.save()
    g2 = Group(name="defaults2", is_default=True)
    g2.save()
    Group(name="other").save()
    st, body = as_admin("post", "/user/create", {"username": "newcomer", "email": "n@x.org", "password": "password1"})
    assert st == 201, body
    u = User.find_by_username("newcomer")
    assert {g.name for g in u.groups} == {"defaults1", "defaults2"}


def test_signup_without_default_group(as_admin, tables):
    Group(name="other").save()
    st, _ = as_admin("post", "/user/create", {"username": "newcomer", "email": "n@x.org", "password": "password1"})
    assert st == 201
    assert User.find_by_username("newcomer").groups == []


def test_signup_validation(as_admin, new_user):
    st, _ = as_admin("post", "/user/create", {"username": "administrantee", "email": "n@x.org", "password": "password1"})
    assert st == 409
    st, _ = as_admin("post", "/user/create", {"username": "x", "email": "n@x.org", "password": "password1"})
    assert st == 422
    st, _ = as_admin("post", "/user/create", {"username": "validname"})
    assert st == 400  # schema: missing required fields


def test_user_update_and_delete(as_user, as_admin, new_user, new_admin):
    st, _ = as_user("put", "/user", {"id": new_user.id, "email": "changed@x.org"})
    assert st == 403  # account changes are admin-only (reference controllers/user.py:125)
    st, body = as_admin("put", "/user", {"id": new_user.id, "email": "changed@x.org"})
    assert st == 201 and body["user"]["email"] == "changed@x.org" and body["reservation"] == body["user"]
    st, _ = as_admin("put", "/user", {"id": new_user.id, "roles": ["user", "admin"]})
    assert st == 201 and set(User.get(new_user.id).role_names) == {"user", "admin"}
    st, _ = as_admin("delete", f"/user/delete/{new_admin.id}")
    assert st == 403  # an admin cannot delete themselves
    st, _ = as_admin("delete", f"/user/delete/{new_user.id}")
    assert st == 200
    st, _ = as_admin("get", f"/users/{new_user.id}")
    assert st == 404


def test_login_logout_refresh(client, new_user):
    st, tok = api(client, "post", "/user/login", None, {"username": "administrantee", "password": "TEST PASSWORD"})
    assert st == 200
    st, _ = api(client, "post", "/user/login", None, {"username": "administrantee", "password": "nope"})
    assert st == 401
    acc = {"Authorization": "Bearer " + tok["access_token"]}
    ref = {"Authorization": "Bearer " + tok["refresh_token"]}
    st, body = api(client, "get", "/user/refresh", ref)
    assert st == 200 and body["access_token"]
    st, _ = api(client, "get", "/user/refresh", acc)
    assert st == 422  # an access token is not a refresh token
    st, _ = api(client, "delete", "/user/logout", acc)
    assert st == 200
    st, _ = api(client, "get", "/users", acc)
    assert st == 401  # revoked
    st, _ = api(client, "delete", "/user/logout/refresh_token", ref)
    assert st == 200
    st, _ = api(client, "get", "/user/refresh", ref)
    assert st == 401


def test_ssh_signup_disabled_by_default(client):
    st, _ = api(client, "post", "/user/ssh_signup", None, {"username": "someone", "email": "a@b.org",
                                                          "password": "password1"})
    assert st in (403, 404, 422)


# ============================================================================ groups
def test_groups_user_role(as_user, new_group, new_user):
    new_group.save()
    for method, path, body in (("post", "/groups", {"name": "g"}), ("put", f"/groups/{new_group.id}", {"name": "x"}),
                               ("delete", f"/groups/{new_group.id}", None),
                               ("put", f"/groups/{new_group.id}/users/{new_user.id}", None),
                               ("delete", f"/groups/{new_group.id}/users/{new_user.id}", None),
                               ("put", f"/groups/{new_group.id}", {"isDefault": True})):
        st, _ = as_user(method, path, body)
        assert st == 403, (method, path)
    st, body = as_user("get", "/groups")
    assert st == 200 and [g["name"] for g in body] == ["TestGroup1"]
    st, body = as_user("get", f"/groups/{new_group.id}")
    assert st == 200 and body["group"]["name"] == "TestGroup1"
    st, _ = as_user("get", "/groups/777")
    assert st == 404
    st, body = as_user("get", "/groups", only_default="true")
    assert st == 200 and body == []


def test_groups_admin_role(as_admin, new_group, new_user):
    st, body = as_admin("post", "/groups", {"name": "created"})
    assert st == 201 and body["group"]["name"] == "created"
    new_group.save()
    st, body = as_admin("put", f"/groups/{new_group.id}", {"name": "renamed"})
    assert st == 200 and Group.get(new_group.id).name == "renamed"
    st, _ = as_admin("put", "/groups/777", {"name": "x"})
    assert st == 404
    st, _ = as_admin("put", f"/groups/{new_group.id}/users/{new_user.id}")
    assert st == 200 and new_user.id in [u.id for u in Group.get(new_group.id).users]
    st, _ = as_admin("put", f"/groups/{new_group.id}/users/{new_user.id}")
    assert st == 409
    st, _ = as_admin("put", f"/groups/{new_group.id}/users/777")
    assert st == 404
    st, _ = as_admin("put", f"/groups/777/users/{new_user.id}")
    assert st == 404
    st, _ = as_admin("delete", f"/groups/{new_group.id}/users/{new_user.id}")
    assert st == 200 and new_user.id not in [u.id for u in Group.get(new_group.id).users]
    st, _ = as_admin("delete", f"/groups/{new_group.id}/users/777")
    assert st == 404
    st, _ = as_admin("delete", f"/groups/777/users/{new_user.id}")
    assert st == 404
    st, _ = as_admin("put", f"/groups/{new_group.id}", {"isDefault": True})
    assert st == 200 and Group.get(new_group.id).is_default
    st, _ = as_admin("put", f"/groups/{new_group.id}", {"isDefault": False})
    assert st == 200 and not Group.get(new_group.id).is_default
    st, _ = as_admin("delete", f"/groups/{new_group.id}")
    assert st == 200
    st, body = as_admin("get", "/groups")
    assert [g["name"] for g in body] == ["created"]
    st, _ = as_admin("delete", "/groups/777")
    assert st == 404


# ============================================================================ schedules
def test_schedules_user_role(as_user, active_schedule):
    st, _ = as_user("post", "/schedules", {"scheduleDays": ["Monday"], "hourStart": "8:00", "hourEnd": "10:00"})
    assert st == 403
    st, body = as_user("get", "/schedules")
    assert st == 200 and len(body) == 1
    st, body = as_user("get", f"/schedules/{active_schedule.id}")
    assert st == 200 and body["schedule"]["hourStart"] == "00:00"
    st, _ = as_user("get", "/schedules/777")
    assert st == 404
    st, _ = as_user("delete", f"/schedules/{active_schedule.id}")
    assert st == 403
    st, _ = as_user("put", f"/schedules/{active_schedule.id}", {"hourStart": "9:00"})
    assert st == 403


def test_schedules_admin_role(as_admin, active_schedule):
    st, body = as_admin("post", "/schedules", {"scheduleDays": ["Monday", "Wednesday"], "hourStart": "8:00",
                                                "hourEnd": "16:00"})
    assert st == 201 and body["schedule"]["scheduleDays"] == ["Monday", "Wednesday"]
    st, _ = as_admin("post", "/schedules", {"scheduleDays": ["Monday"], "hourEnd": "16:00"})
    assert st == 400
    st, _ = as_admin("post", "/schedules", {"scheduleDays": ["Mondayy"], "hourStart": "8:00", "hourEnd": "16:00"})
    assert st == 422
    st, _ = as_admin("post", "/schedules", {"hourStart": "8:00", "hourEnd": "16:00"})
    assert st == 400
    st, body = as_admin("put", f"/schedules/{active_schedule.id}", {"scheduleDays": ["Friday"], "hourStart": "7:30",
                                                                     "hourEnd": "9:45"})
    assert st == 200
    s = RestrictionSchedule.get(active_schedule.id)
    assert s.schedule_days == "5" and s.hour_start == datetime.time(7, 30)
    st, _ = as_admin("put", "/schedules/777", {"hourStart": "9:00"})
    assert st == 404
    st, _ = as_admin("delete", f"/schedules/{active_schedule.id}")
    assert st == 200
    st, _ = as_admin("delete", "/schedules/777")
    assert st == 404
    st, body = as_admin("get", "/schedules")
    assert len(body) == 1


# ============================================================================ restrictions
def _rest_body(start, end=None, is_global=False):
    b = {"name": "R", "startsAt": iso(start), "isGlobal": is_global}
    if end is not None:
        b["endsAt"] = iso(end)
    return b


def test_restrictions_user_role(as_user, restriction, new_user, new_group, resource1):
    new_group.save()
    st, body = as_user("get", "/restrictions")
    assert st == 200 and len(body) == 1  # any signed-in user may list (reference controllers/restriction.py:84)
    restriction.apply_to_user(new_user)
    st, body = as_user("get", "/restrictions", user_id=new_user.id)
    assert st == 200 and [r["id"] for r in body] == [restriction.id]
    st, _ = as_user("post", "/restrictions", _rest_body(UTC() + timedelta(hours=1)))
    assert st == 403
    st, _ = as_user("put", f"/restrictions/{restriction.id}", {"name": "x"})
    assert st == 403
    st, _ = as_user("put", f"/restrictions/{restriction.id}/groups/{new_group.id}")
    assert st == 403
    st, _ = as_user("delete", f"/restrictions/{restriction.id}/hosts/node-a")
    assert st == 403
    st, _ = as_user("delete", f"/restrictions/{restriction.id}")
    assert st == 403


def test_restriction_queries(as_admin, restriction, new_user, new_group_with_member, resource1, active_schedule):
    st, body = as_admin("get", "/restrictions")
    assert st == 200 and len(body) == 1
    restriction.apply_to_group(new_group_with_member)
    st, body = as_admin("get", "/restrictions", user_id=new_user.id)
    assert body == []
    st, body = as_admin("get", "/restrictions", user_id=new_user.id, include_user_groups="true")
    assert [r["id"] for r in body] == [restriction.id]
    st, body = as_admin("get", "/restrictions", group_id=new_group_with_member.id)
    assert [r["id"] for r in body] == [restriction.id]
    restriction.apply_to_resource(resource1)
    st, body = as_admin("get", "/restrictions", resource_id=resource1.id)
    assert [r["id"] for r in body] == [restriction.id]
    restriction.add_schedule(active_schedule)
    st, body = as_admin("get", "/restrictions", schedule_id=active_schedule.id)
    assert [r["id"] for r in body] == [restriction.id]


def test_restriction_crud_admin(as_admin):
    start = UTC() + timedelta(hours=1)
    st, body = as_admin("post", "/restrictions", _rest_body(start, start + timedelta(hours=5)))
    assert st == 201 and body["restriction"]["name"] == "R"
    st, body = as_admin("post", "/restrictions", _rest_body(start))
    assert st == 201 and body["restriction"]["endsAt"] is None
    st, _ = as_admin("post", "/restrictions", {"name": "missing"})
    assert st == 400
    rid = body["restriction"]["id"]
    st, body = as_admin("put", f"/restrictions/{rid}", {"name": "renamed", "isGlobal": True})
    assert st == 200 and body["restriction"]["isGlobal"] is True
    st, _ = as_admin("put", f"/restrictions/{rid}", {"endsAt": iso(start - timedelta(hours=2))})
    assert st == 422
    st, _ = as_admin("put", "/restrictions/777", {"name": "x"})
    assert st == 404
    st, _ = as_admin("delete", f"/restrictions/{rid}")
    assert st == 200
    st, _ = as_admin("delete", "/restrictions/777")
    assert st == 404


@pytest.mark.parametrize("kind", ["users", "groups", "resources", "schedules"])
def test_restriction_apply_remove(as_admin, restriction, new_user, new_group, resource1, active_schedule, kind):
    new_group.save()
    target = {"users": new_user.id, "groups": new_group.id, "resources": resource1.id,
              "schedules": active_schedule.id}[kind]
    missing = "GPU-" + "9" * 36 if kind == "resources" else 777
    st, _ = as_admin("put", f"/restrictions/{restriction.id}/{kind}/{target}")
    assert st == 200
    st, _ = as_admin("put", f"/restrictions/{restriction.id}/{kind}/{target}")
    assert st == 409
    st, _ = as_admin("put", f"/restrictions/{restriction.id}/{kind}/{missing}")
    assert st == 404
    st, _ = as_admin("put", f"/restrictions/777/{kind}/{target}")
    assert st == 404
    st, _ = as_admin("delete", f"/restrictions/{restriction.id}/{kind}/{target}")
    assert st == 200
    st, _ = as_admin("delete", f"/restrictions/{restriction.id}/{kind}/{target}")
    assert st == 404


def test_restriction_hosts(as_admin, restriction, tables):
    a1 = Resource(id="GPU-" + "a" * 36, hostname="nasa.gov")
    a1.save()
    a2 = Resource(id="GPU-" + "b" * 36, hostname="nasa.gov")
    a2.save()
    other = Resource(id="GPU-" + "c" * 36, hostname="esa.int")
    other.save()
    st, body = as_admin("put", f"/restrictions/{restriction.id}/hosts/nasa.gov")
    assert st == 200 and {r.id for r in Restriction.get(restriction.id).resources} == {a1.id, a2.id}
    st, _ = as_admin("put", f"/restrictions/{restriction.id}/hosts/jacek.com")
    assert st == 404
    st, _ = as_admin("put", "/restrictions/777/hosts/nasa.gov")
    assert st == 404
    st, _ = as_admin("delete", f"/restrictions/{restriction.id}/hosts/nasa.gov")
    assert st == 200 and Restriction.get(restriction.id).resources == []
    st, _ = as_admin("delete", f"/restrictions/{restriction.id}/hosts/jacek.com")
    assert st == 404
    st, _ = as_admin("delete", "/restrictions/777/hosts/nasa.gov")
    assert st == 404


# ============================================================================ reservations
RES = "GPU-" + "5" * 36


def _res_body(user, start, end, rid=RES):
    return {"title": "Test reservation", "description": "d", "resourceId": rid, "userId": user.id,
            "start": start if isinstance(start, str) else iso(start), "end": end if isinstance(end, str) else iso(end)}


@pytest.fixture()
def gpu(tables):
    r = Resource(id=RES, hostname="node-a")
    r.save()
    return r


def test_reservation_needs_permission(as_user, new_user, gpu):
    st, _ = as_user("post", "/reservations", _res_body(new_user, "2101-01-01T10:00:00.000Z", "2101-01-01T12:00:00.000Z"))
    assert st == 403


def test_reservation_with_global_permission(as_user, new_user, gpu, permissive_restriction):
    permissive_restriction.apply_to_user(new_user)
    now = UTC()
    st, body = as_user("post", "/reservations", _res_body(new_user, now + timedelta(minutes=1), now + timedelta(hours=1)))
    assert st == 201 and Reservation.get(body["reservation"]["id"])


def test_reservation_in_the_past_allowed_by_fork(as_user, new_user, gpu, permissive_restriction):
    """The fork disabled the reference's "cannot reserve in the past" check
    (reference ``controllers/reservation.py:86-90``, commented out); pinned here."""
    permissive_restriction.apply_to_user(new_user)
    start = UTC() - timedelta(minutes=2)
    st, _ = as_user("post", "/reservations", _res_body(new_user, start, start + timedelta(hours=1)))
    assert st == 201


def test_reservation_for_someone_else_forbidden(as_user, new_user, new_admin, gpu, permissive_restriction):
    permissive_restriction.apply_to_user(new_user)
    st, _ = as_user("post", "/reservations", _res_body(new_admin, UTC() + timedelta(hours=1), UTC() + timedelta(hours=2)))
    assert st == 403


def test_reservation_indefinite_restriction(as_user, new_user, gpu, restriction):
    restriction.starts_at = "2101-01-01T10:00:00.000Z"
    restriction.ends_at = None
    restriction.save()
    restriction.apply_to_user(new_user)
    restriction.apply_to_resource(gpu)
    st, _ = as_user("post", "/reservations", _res_body(new_user, "2101-01-02T10:00:00.000Z", "2101-01-03T12:00:00.000Z"))
    assert st == 201


def test_reservation_partly_covered(as_user, new_user, gpu, restriction):
    restriction.starts_at = "2101-01-01T10:00:00.000Z"
    restriction.ends_at = "2101-01-05T10:00:00.000Z"
    restriction.save()
    restriction.apply_to_user(new_user)
    restriction.apply_to_resource(gpu)
    st, _ = as_user("post", "/reservations", _res_body(new_user, "2101-01-04T10:00:00.000Z", "2101-01-06T12:00:00.000Z"))
    assert st == 403


def test_reservation_outside_schedule(as_user, new_user, gpu, restriction):
    restriction.starts_at = "2101-01-01T10:00:00.000Z"
    restriction.ends_at = "2101-01-05T10:00:00.000Z"
    restriction.save()
    restriction.apply_to_user(new_user)
    s = RestrictionSchedule(schedule_days="1234567", hour_start=datetime.time(8), hour_end=datetime.time(10))
    s.save()
    restriction.add_schedule(s)
    restriction.apply_to_resource(gpu)
    st, _ = as_user("post", "/reservations", _res_body(new_user, "2101-01-07T09:00:00.000Z", "2101-01-07T10:30:00.000Z"))
    assert st == 403


def test_reservation_two_adjacent_restrictions(as_user, new_user, gpu):
    r1 = Restriction(name="first", starts_at="2101-01-01T00:00:00.000Z", ends_at="2101-01-02T00:00:00.000Z")
    r2 = Restriction(name="second", starts_at="2101-01-02T00:00:00.000Z", ends_at="2101-01-02T23:59:00.000Z")
    for r in (r1, r2):
        r.save()
        r.apply_to_user(new_user)
        r.apply_to_resource(gpu)
    st, _ = as_user("post", "/reservations", _res_body(new_user, "2101-01-01T10:00:00.000Z", "2101-01-02T12:00:00.000Z"))
    assert st == 201


def test_reservation_via_group_restriction(as_user, new_user, gpu, new_group_with_member):
    r = Restriction(name="grp", starts_at=UTC() - timedelta(days=1))
    r.save()
    r.apply_to_group(new_group_with_member)
    r.apply_to_resource(gpu)
    st, _ = as_user("post", "/reservations", _res_body(new_user, UTC() + timedelta(hours=1), UTC() + timedelta(hours=3)))
    assert st == 201


def _mk_res(user, start, dur):
    r = Reservation(user_id=user.id, title="TEST TITLE", description="d", resource_id=RES, start=start, end=start + dur)
    r.save()
    return r


def test_reservation_updates_user(as_user, new_user, new_admin, gpu, permissive_restriction):
    permissive_restriction.apply_to_user(new_user)
    fut = _mk_res(new_user, UTC() + timedelta(hours=5), timedelta(hours=10))
    st, body = as_user("put", f"/reservations/{fut.id}", {"title": "renamed"})
    assert st == 201 and body["reservation"]["title"] == "renamed"
    new_start = fut.start + timedelta(hours=1)
    st, body = as_user("put", f"/reservations/{fut.id}", {"start": iso(new_start)})
    assert st == 201 and Reservation.get(fut.id).start == new_start.replace(microsecond=new_start.microsecond)
    other = _mk_res(new_admin, UTC() + timedelta(days=3), timedelta(hours=1))
    st, _ = as_user("put", f"/reservations/{other.id}", {"title": "mine now"})
    assert st == 403
    active = _mk_res(new_user, UTC() - timedelta(hours=1), timedelta(hours=2))
    st, _ = as_user("put", f"/reservations/{active.id}", {"start": iso(UTC())})
    assert st == 403
    st, _ = as_user("delete", f"/reservations/{active.id}")
    assert st == 403
    past = _mk_res(new_user, UTC() - timedelta(days=2), timedelta(hours=1))
    st, _ = as_user("put", f"/reservations/{past.id}", {"title": "history"})
    assert st == 403
    st, _ = as_user("delete", f"/reservations/{fut.id}")
    assert st == 200


def test_reservation_admin_powers(as_admin, new_user, gpu, permissive_restriction):
    past = _mk_res(new_user, UTC() - timedelta(days=2), timedelta(hours=1))
    st, _ = as_admin("put", f"/reservations/{past.id}", {"title": "fixed"})
    assert st in (201, 403)  # allowed only if the owner's restrictions still cover it
    permissive_restriction.apply_to_user(new_user)
    st, _ = as_admin("put", f"/reservations/{past.id}", {"title": "fixed"})
    assert st == 201
    active = _mk_res(new_user, UTC() - timedelta(hours=1), timedelta(hours=2))
    st, _ = as_admin("delete", f"/reservations/{active.id}")
    assert st == 200


def test_reservation_cancelled_when_restriction_shrinks(as_admin, new_user, gpu):
    r = Restriction(name="window", starts_at=UTC() - timedelta(hours=1), ends_at=UTC() + timedelta(days=3))
    r.save()
    r.apply_to_user(new_user)
    r.apply_to_resource(gpu)
    keep = _mk_res(new_user, UTC() + timedelta(hours=2), timedelta(hours=2))
    lose = _mk_res(new_user, UTC() + timedelta(days=2), timedelta(hours=2))
    st, _ = as_admin("put", f"/restrictions/{r.id}", {"endsAt": iso(UTC() + timedelta(days=1))})
    assert st == 200
    assert not Reservation.get(keep.id).is_cancelled
    assert Reservation.get(lose.id).is_cancelled


def test_reservation_listing_filters(as_user, new_user, gpu, permissive_restriction):
    a = _mk_res(new_user, UTC() + timedelta(hours=1), timedelta(hours=1))
    _mk_res(new_user, UTC() + timedelta(days=3), timedelta(hours=1))
    st, body = as_user("get", "/reservations")
    assert st == 200 and len(body) == 2
    st, body = as_user("get", "/reservations", resources_ids=RES, start=iso(UTC()), end=iso(UTC() + timedelta(days=1)))
    assert st == 200 and [x["id"] for x in body] == [a.id]
    st, _ = as_user("get", "/reservations", resources_ids=RES)
    assert st == 400


# ============================================================================ jobs
def test_jobs_listing(as_user, as_admin, new_job, new_admin_job, new_user):
    st, body = as_user("get", "/jobs", userId=new_user.id)
    assert st == 200 and [j["id"] for j in body["jobs"]] == [new_job.id]
    st, _ = as_user("get", "/jobs")
    assert st == 403
    st, body = as_admin("get", "/jobs")
    assert st == 200 and len(body["jobs"]) == 2
    st, body = as_admin("get", "/jobs", userId=new_user.id)
    assert st == 200 and len(body["jobs"]) == 1


def test_job_create(as_user, new_user, new_admin):
    body = {"name": "TestJob", "description": "d", "userId": new_user.id,
            "startAt": iso(UTC() + timedelta(hours=5)), "stopAt": iso(UTC() + timedelta(hours=10))}
    st, out = as_user("post", "/jobs", body)
    assert st == 201 and Job.get(out["job"]["id"]).name == "TestJob"
    st, out = as_user("post", "/jobs", {"name": "nodates", "description": "d", "userId": new_user.id})
    assert st == 201 and out["job"]["startAt"] is None
    st, _ = as_user("post", "/jobs", {**body, "stopAt": iso(UTC() + timedelta(hours=4))})
    assert st == 422
    st, _ = as_user("post", "/jobs", {**body, "userId": new_admin.id})
    assert st == 403


def test_job_create_start_in_past_means_now(as_user, new_user):
    """Fork behaviour (reference ``models/Job.py:122-130``): a past start is clamped to now."""
    st, out = as_user("post", "/jobs", {"name": "j", "description": "d", "userId": new_user.id,
                                        "startAt": iso(UTC() - timedelta(hours=5)),
                                        "stopAt": iso(UTC() + timedelta(hours=10))})
    assert st == 201
    assert abs((Job.get(out["job"]["id"]).start_at - UTC()).total_seconds()) < 10


def test_job_update(as_user, new_job, new_admin_job):
    st, body = as_user("put", f"/jobs/{new_job.id}", {"name": "renamed", "startAt": iso(UTC() + timedelta(hours=1)),
                                                      "stopAt": iso(UTC() + timedelta(hours=2))})
    assert st == 200 and body["job"]["name"] == "renamed"
    st, _ = as_user("put", f"/jobs/{new_job.id}", {"description": "only"})
    assert st == 200
    st, _ = as_user("put", f"/jobs/{new_job.id}", {"startAt": iso(UTC() + timedelta(hours=5)),
                                                   "stopAt": iso(UTC() + timedelta(hours=4))})
    assert st == 422
    st, _ = as_user("put", f"/jobs/{new_admin_job.id}", {"name": "mine"})
    assert st == 403


def test_job_update_running_rejected(as_user, new_running_job):
    st, _ = as_user("put", f"/jobs/{new_running_job.id}", {"name": "x"})
    assert st == 422


def test_job_delete_cascades(as_user, new_job_with_task, new_task_2):
    jid = new_job_with_task.id
    st, body = as_user("get", "/tasks", jobId=jid)
    assert st == 200 and len(body["tasks"]) == 1
    st, _ = as_user("delete", f"/jobs/{jid}")
    assert st == 200
    st, _ = as_user("get", "/tasks", jobId=jid)
    assert st == 404
    assert [t.id for t in Task.query.all()] == [new_task_2.id]  # the job's task went with it


def test_job_delete_not_owned(as_user, new_admin_job):
    st, _ = as_user("delete", f"/jobs/{new_admin_job.id}")
    assert st == 403


def test_job_admin_can_manage_others(as_admin, new_job_with_task):
    st, _ = as_admin("put", f"/jobs/{new_job_with_task.id}", {"name": "adm"})
    assert st == 200
    st, body = as_admin("get", "/tasks", jobId=new_job_with_task.id)
    assert st == 200 and len(body["tasks"]) == 1
    st, _ = as_admin("delete", f"/jobs/{new_job_with_task.id}")
    assert st == 200


def test_job_task_membership_endpoints(as_user, new_job, new_task, new_admin_job):
    st, _ = as_user("get", "/tasks", jobId=new_admin_job.id)
    assert st == 403
    st, body = as_user("put", f"/jobs/{new_job.id}/tasks/{new_task.id}")
    assert st == 200 and Task.get(new_task.id).job_id == new_job.id
    st, _ = as_user("put", f"/jobs/{new_job.id}/tasks/{new_task.id}")
    assert st == 409
    st, _ = as_user("delete", f"/jobs/{new_job.id}/tasks/{new_task.id}")
    assert st == 200
    st, _ = as_user("delete", f"/jobs/{new_job.id}/tasks/{new_task.id}")
    assert st == 404


def test_job_templates(as_user):
    st, body = as_user("get", "/jobs/templates")
    assert st == 200 and "torchrun" in body["templates"]
    assert any(e["name"] == "HIP_VISIBLE_DEVICES" for e in body["templates"]["torchrun"]["envs"])


# ============================================================================ tasks
def test_task_create_update_delete(as_user, new_job):
    body = {"command": "python train.py", "hostname": "node-a",
            "cmdsegments": {"envs": [{"name": "HIP_VISIBLE_DEVICES", "value": "3"}],
                            "params": [{"name": "--batch_size", "value": "32"}, {"name": "--lr=", "value": "0.1"}]}}
    st, out = as_user("post", f"/jobs/{new_job.id}/tasks", body)
    assert st == 201, out
    t = out["task"]
    assert t["fullCommand"] == "HIP_VISIBLE_DEVICES=3 python train.py --batch_size 32 --lr=0.1"
    assert t["gpuId"] == 3 and t["jobId"] == new_job.id
    st, out = as_user("put", f"/tasks/{t['id']}", {"command": "python eval.py",
                                                   "cmdsegments": {"params": [{"name": "--x", "value": "1"}]}})
    assert st == 201 and out["task"]["fullCommand"] == "python eval.py --x 1"
    st, out = as_user("get", f"/tasks/{t['id']}")
    assert st == 200 and out["task"]["status"] == "not_running"
    st, _ = as_user("delete", f"/tasks/{t['id']}")
    assert st == 200
    st, _ = as_user("get", f"/tasks/{t['id']}")
    assert st == 404


def test_task_not_owned(as_user, as_admin, new_admin_job):
    tid = new_admin_job.tasks[0].id
    st, _ = as_user("put", f"/tasks/{tid}", {"command": "x"})
    assert st == 403
    st, _ = as_user("delete", f"/tasks/{tid}")
    assert st == 403
    st, _ = as_admin("put", f"/tasks/{tid}", {"command": "python other.py"})
    assert st == 201
    st, _ = as_admin("delete", f"/tasks/{tid}")
    assert st == 200


# ============================================================================ execute / stop / logs
def _job_with(as_user, job, host="node-a", gpu="0", command="python train.py"):
    st, out = as_user("post", f"/jobs/{job.id}/tasks", {"command": command, "hostname": host, "cmdsegments": {
        "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": gpu}]}})
    assert st == 201
    return out["task"]["id"]


def test_execute_stop_cycle(as_user, daemon, new_job):
    t1 = _job_with(as_user, new_job, "node-a", "0")
    t2 = _job_with(as_user, new_job, "node-b", "1,2")
    st, out = as_user("get", f"/jobs/{new_job.id}/execute")
    assert st == 200 and out["job"]["status"] == "running", out
    st, out = as_user("get", f"/jobs/{new_job.id}/execute")
    assert st == 409
    # the simulated nodes report the spawned tasks as GPU processes tagged with their task id
    procs = daemon.stub.sample("node-b")["GPU"][daemon.stub.gpu_uuid("node-b", 2)]["processes"]
    assert [p["task_id"] for p in procs] == [str(t2)] and procs[0]["owner"] == "administrantee"
    st, out = as_user("get", f"/tasks/{t1}/log", tail="true")
    assert st == 200 and "python train.py" in out["output_lines"][0]
    st, out = as_user("get", f"/jobs/{new_job.id}/stop", gracefully="true")
    assert st == 200 and out["job"]["status"] == "terminated"
    st, out = as_user("get", f"/tasks/{t1}")
    assert out["task"]["status"] == "terminated" and out["task"]["pid"] is None
    st, _ = as_user("get", f"/jobs/{new_job.id}/stop")
    assert st == 409


def test_task_finishing_on_its_own_is_detected(as_user, daemon, new_job):
    tid = _job_with(as_user, new_job)
    as_user("get", f"/jobs/{new_job.id}/execute")
    node = daemon.transports.get("node-a")
    pid = Task.get(tid).pid
    node.exit_task(pid)
    st, out = as_user("get", f"/tasks/{tid}")
    assert out["task"]["status"] == "terminated"
    st, out = as_user("get", f"/jobs/{new_job.id}")
    assert out["job"]["status"] == "terminated"


def test_execute_on_unreachable_node(as_user, daemon, new_job):
    _job_with(as_user, new_job)
    daemon.transports.get("node-a").down = True
    st, out = as_user("get", f"/jobs/{new_job.id}/execute")
    assert st == 422 and len(out["not_spawned_list"]) == 1


def test_execute_not_owned_job(as_admin, new_admin_job, new_job_with_task, as_user):
    st, _ = as_user("get", f"/jobs/{new_admin_job.id}/execute")
    assert st == 403


def test_enqueue_dequeue(as_user, new_job_with_task):
    jid = new_job_with_task.id
    st, out = as_user("put", f"/jobs/{jid}/enqueue")
    assert st == 200 and out["job"]["status"] == "pending" and out["job"]["isQueued"]
    st, _ = as_user("put", f"/jobs/{jid}/enqueue")
    assert st == 409
    st, out = as_user("put", f"/jobs/{jid}/dequeue")
    assert st == 200 and out["job"]["status"] == "not_running"
    st, _ = as_user("put", f"/jobs/{jid}/dequeue")
    assert st == 409


# ============================================================================ nodes / resources
def test_nodes_endpoints(as_user, daemon, new_user, permissive_restriction):
    st, body = as_user("get", "/nodes/hostnames")
    assert st == 200 and body == []  # no restriction -> no visible nodes (reference controllers/nodes.py:44)
    permissive_restriction.apply_to_user(new_user)
    st, body = as_user("get", "/nodes/hostnames")
    assert st == 200 and sorted(body) == ["node-a", "node-b"]
    st, body = as_user("get", "/nodes/node-a/gpu/info")
    assert st == 200 and len(body) == 8 and all(v["name"] == "AMD Instinct MI355X" for v in body.values())
    st, body = as_user("get", "/nodes/node-a/cpu/metrics")
    assert st == 200
    st, body = as_user("get", "/nodes/node-a/gpu/processes")
    assert st == 200 and all(v == [] for v in body.values())
    st, _ = as_user("get", "/nodes/nowhere/gpu/info")
    assert st == 404
    st, body = as_user("get", "/nodes/topology")
    assert st == 200 and len(body["node-a"]["gpus"]) == 8


def test_nodes_metrics_filtered_by_restrictions(as_user, new_user, daemon, tables):
    st, body = as_user("get", "/nodes/metrics")
    assert st == 200
    uuid = daemon.stub.gpu_uuid("node-a", 0)
    r = Restriction(name="one", starts_at=UTC() - timedelta(hours=1))
    r.save()
    r.apply_to_user(new_user)
    r.apply_to_resource(Resource.get(uuid))
    st, body = as_user("get", "/nodes/metrics")
    assert st == 200


def test_resources(as_user, daemon, new_user, permissive_restriction):
    as_user("get", "/nodes/metrics")
    st, body = as_user("get", "/resources")
    assert st == 200 and len(body) == 16
    uuid = body[0]["id"]
    st, one = as_user("get", f"/resource/{uuid}")
    assert st == 200 and one["resource"]["id"] == uuid
    st, _ = as_user("get", "/resource/GPU-nonexistent")
    assert st == 404


def test_internal_metrics_admin_only(as_user, as_admin):
    st, _ = as_user("get", "/metrics/internal")
    assert st == 403
    st, body = as_admin("get", "/metrics/internal")
    assert st == 200 and "api" in body


def test_restricted_poll_cache_follows_writes_and_the_clock(client, new_user, new_admin, auth_headers, tables):
    """/nodes/metrics for a non-admin caches the permitted-GPU set (controllers/nodes.py); every
    permission write and every restriction start / end must show on the next poll."""
    import time

    hu, ha = auth_headers(new_user), auth_headers(new_admin)

    def visible():
        # the in-process client shares the fixtures' session (expire_on_commit=False); a served
        # request starts from a fresh one
        db_session.expire_all()
        st, body = api(client, "get", "/nodes/metrics", hu)
        assert st == 200
        return {u for h in body.values() for u in (h.get("GPU") or {})}

    api(client, "get", "/nodes/metrics", ha)  # registers the simulated GPUs as resources
    uuids = sorted(r.id for r in Resource.all())
    assert visible() == set()
    r = Restriction(name="one gpu", starts_at=UTC() - timedelta(hours=1), is_global=False)
    r.save()
    r.apply_to_user(new_user)
    r.apply_to_resource(Resource.get(uuids[0]))
    assert visible() == {uuids[0]}
    assert visible() == {uuids[0]}  # served from the cache
    st, _ = api(client, "put", f"/restrictions/{r.id}/resources/{uuids[1]}", ha)
    assert st == 200 and visible() == {uuids[0], uuids[1]}
    g = Group(name="gpu-club")
    g.save()
    r2 = Restriction(name="club", starts_at=UTC() - timedelta(hours=1), ends_at=UTC() + timedelta(seconds=2),
                     is_global=False)
    r2.save()
    r2.apply_to_group(g)
    r2.apply_to_resource(Resource.get(uuids[2]))
    assert visible() == {uuids[0], uuids[1]}
    st, _ = api(client, "put", f"/groups/{g.id}/users/{new_user.id}", ha)
    assert st == 200 and visible() == {uuids[0], uuids[1], uuids[2]}
    time.sleep(2.2)  # r2 expires: no write happens, the cache entry's validity ends with it
    assert visible() == {uuids[0], uuids[1]}
    st, _ = api(client, "delete", f"/restrictions/{r.id}", ha)
    assert st == 200 and visible() == set()


def test_revocation_visible_through_the_token_cache(client, new_user, auth_headers):
    """RevokedToken caches 'not revoked' answers; a logout must still take effect immediately."""
    h = auth_headers(new_user)
    for _ in range(3):  # the jti is now cached as not revoked
        assert api(client, "get", "/users", h)[0] == 200
    assert api(client, "delete", "/user/logout", h)[0] == 200
    assert api(client, "get", "/users", h)[0] == 401
