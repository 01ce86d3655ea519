"""Scenario-for-scenario counterparts of the reference controller tests
(``tests/functional/controllers/test_*_controller{,_superuser}.py``, 127 functions).

One class per reference module, one method per reference function with the same name, so the
mapping in PARITY.md is mechanical.  The reference patches the JWT decorators and calls the view
functions; here every request carries a real token (``as_user`` = the unprivileged role,
``as_admin`` = the superuser role) and passes the OpenAPI validator, which also checks every
response body against the document.  Where this fork deliberately differs (documented in
PARITY.md) the assertion says so.
"""
import datetime
from datetime import timedelta

import pytest

from tensorhive_fixed_amd.database import db_session
from tensorhive_fixed_amd.models.orm import (CommandSegment, Group, Job, Reservation, Resource, Restriction,
                                             RestrictionSchedule, Task, User)
from tests.helpers import api

UTC = datetime.datetime.utcnow
FMT = "%Y-%m-%dT%H:%M:%S.%fZ"
GPU = "GPU-" + "0123456789" * 3 + "012345"  # a 40-character resource id


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


@pytest.fixture()
def granted(new_user, new_admin, permissive_restriction):
    """The reference's permissive_restriction fixture: global, open-ended, applied to the user."""
    permissive_restriction.apply_to_user(new_user)
    permissive_restriction.apply_to_user(new_admin)
    return permissive_restriction


def _gpu(uuid=GPU, host="node-a"):
    r = Resource(id=uuid, hostname=host)
    r.save()
    return r


# ================================================================= test_group_controller.py
class TestGroupController:
    def test_create_group_unprivileged(self, as_user):
        assert as_user("post", "/groups", {"name": "TestGroup"})[0] == 403

    def test_update_group_unprivileged(self, as_user, new_group):
        new_group.save()
        assert as_user("put", f"/groups/{new_group.id}", {"name": "Modified"})[0] == 403
        assert Group.get(new_group.id).name == "TestGroup1"

    def test_delete_group_unprivileged(self, as_user, new_group):
        new_group.save()
        assert as_user("delete", f"/groups/{new_group.id}")[0] == 403
        assert Group.get(new_group.id) is not None

    def test_add_user_to_a_group_unprivileged(self, as_user, new_group, new_user):
        new_group.save()
        assert as_user("put", f"/groups/{new_group.id}/users/{new_user.id}")[0] == 403
        assert new_user not in Group.get(new_group.id).users

    def test_remove_user_from_a_group_unprivileged(self, as_user, new_group_with_member, new_user):
        assert as_user("delete", f"/groups/{new_group_with_member.id}/users/{new_user.id}")[0] == 403
        assert new_user in Group.get(new_group_with_member.id).users

    def test_set_group_as_a_default_unprivileged(self, as_user, new_group):
        new_group.save()
        assert as_user("put", f"/groups/{new_group.id}", {"isDefault": True})[0] == 403
        assert not Group.get(new_group.id).is_default

    def test_mark_default_group_as_non_default_unprivileged(self, as_user, new_group):
        new_group.is_default = True
        new_group.save()
        assert as_user("put", f"/groups/{new_group.id}", {"isDefault": False})[0] == 403
        assert Group.get(new_group.id).is_default

    def test_get_list_of_groups(self, as_user, new_group):
        new_group.save()
        Group(name="Second").save()
        st, body = as_user("get", "/groups")
        assert st == 200 and len(body) == 2

    def test_get_list_of_groups_one_group_returned(self, as_user, new_group):
        new_group.save()
        st, body = as_user("get", "/groups")
        assert st == 200 and len(body) == 1 and body[0]["name"] == "TestGroup1"

    def test_get_group_by_id(self, as_user, new_group):
        new_group.save()
        st, body = as_user("get", f"/groups/{new_group.id}")
        assert st == 200 and body["group"]["id"] == new_group.id

    def test_get_group_by_id_that_doesnt_exist(self, as_user):
        assert as_user("get", "/groups/777")[0] == 404

    def test_get_default_groups(self, as_user, new_group):
        new_group.is_default = True
        new_group.save()
        Group(name="NotDefault").save()
        st, body = as_user("get", "/groups", only_default="true")
        assert st == 200 and [g["id"] for g in body] == [new_group.id]

    def test_get_default_groups_when_no_default_group_exists(self, as_user, new_group):
        new_group.save()
        st, body = as_user("get", "/groups", only_default="true")
        assert st == 200 and body == []


# ================================================================= test_group_controller_superuser.py
class TestGroupControllerSuperuser:
    def test_create_group(self, as_admin):
        st, body = as_admin("post", "/groups", {"name": "TestGroup"})
        assert st == 201 and Group.get(body["group"]["id"]).name == "TestGroup"

    def test_update_group(self, as_admin, new_group):
        new_group.save()
        st, body = as_admin("put", f"/groups/{new_group.id}", {"name": "Modified"})
        assert st == 200 and body["group"]["name"] == "Modified" and Group.get(new_group.id).name == "Modified"

    def test_update_group_that_doesnt_exist(self, as_admin):
        assert as_admin("put", "/groups/777", {"name": "Modified"})[0] == 404

    def test_delete_group(self, as_admin, new_group):
        new_group.save()
        assert as_admin("delete", f"/groups/{new_group.id}")[0] == 200
        with pytest.raises(Exception):
            Group.get(new_group.id)

    def test_delete_group_that_doesnt_exist(self, as_admin):
        assert as_admin("delete", "/groups/777")[0] == 404

    def test_add_user_to_a_group(self, as_admin, new_group, new_user):
        new_group.save()
        st, body = as_admin("put", f"/groups/{new_group.id}/users/{new_user.id}")
        assert st == 200 and new_user in Group.get(new_group.id).users
        assert [u["id"] for u in body["group"]["users"]] == [new_user.id]

    def test_remove_user_from_a_group(self, as_admin, new_group_with_member, new_user):
        st, body = as_admin("delete", f"/groups/{new_group_with_member.id}/users/{new_user.id}")
        assert st == 200 and new_user not in Group.get(new_group_with_member.id).users and body["group"]["users"] == []

    def test_add_nonexistent_user_to_a_group(self, as_admin, new_group):
        new_group.save()
        assert as_admin("put", f"/groups/{new_group.id}/users/777")[0] == 404

    def test_add_user_to_nonexistent_group(self, as_admin, new_user):
        assert as_admin("put", f"/groups/777/users/{new_user.id}")[0] == 404

    def test_remove_nonexistent_user_from_a_group(self, as_admin, new_group):
        new_group.save()
        assert as_admin("delete", f"/groups/{new_group.id}/users/777")[0] == 404

    def test_remove_user_from_a_nonexistent_group(self, as_admin, new_user):
        assert as_admin("delete", f"/groups/777/users/{new_user.id}")[0] == 404

    def test_set_group_as_a_default(self, as_admin, new_group):
        new_group.save()
        st, body = as_admin("put", f"/groups/{new_group.id}", {"isDefault": True})
        assert st == 200 and body["group"]["isDefault"] is True and Group.get(new_group.id).is_default

    def test_mark_default_group_as_non_default(self, as_admin, new_group):
        new_group.is_default = True
        new_group.save()
        st, body = as_admin("put", f"/groups/{new_group.id}", {"isDefault": False})
        assert st == 200 and body["group"]["isDefault"] is False and not Group.get(new_group.id).is_default


# ================================================================= test_job_controller.py
class TestJobController:
    def test_get_all_jobs(self, as_user, new_user, new_job, new_admin_job):
        st, body = as_user("get", "/jobs", userId=new_user.id)
        assert st == 200 and len(body["jobs"]) == 1

    def test_create_job(self, as_user, new_user):
        st, body = as_user("post", "/jobs", {"name": "job", "description": "d", "userId": new_user.id,
                                             "startAt": iso(UTC() + timedelta(hours=5)),
                                             "stopAt": iso(UTC() + timedelta(hours=10))})
        assert st == 201 and body["job"]["name"] == "job" and Job.get(body["job"]["id"]) is not None

    def test_create_job_without_dates(self, as_user, new_user):
        st, body = as_user("post", "/jobs", {"name": "job", "description": "d", "userId": new_user.id})
        assert st == 201 and body["job"]["startAt"] is None and body["job"]["stopAt"] is None

    def test_create_job_in_the_past(self, as_user, new_user):
        # fork: a start in the past means "now" (reference models/Job.py:122-130 clamps it too)
        st, body = as_user("post", "/jobs", {"name": "job", "description": "d", "userId": new_user.id,
                                             "startAt": iso(UTC() - timedelta(hours=5))})
        assert st == 201 and abs((Job.get(body["job"]["id"]).start_at - UTC()).total_seconds()) < 10

    def test_create_job_that_stops_before_it_starts(self, as_user, new_user):
        st, _ = as_user("post", "/jobs", {"name": "job", "description": "d", "userId": new_user.id,
                                          "startAt": iso(UTC() + timedelta(hours=5)),
                                          "stopAt": iso(UTC() + timedelta(hours=4))})
        assert st == 422

    def test_update_job(self, as_user, new_job):
        st, body = as_user("put", f"/jobs/{new_job.id}", {"name": "new name", "startAt": iso(UTC() + timedelta(hours=5)),
                                                          "stopAt": iso(UTC() + timedelta(hours=6))})
        assert st == 200 and body["job"]["name"] == "new name" and Job.get(new_job.id).name == "new name"

    def test_update_job_without_dates(self, as_user, new_job):
        st, body = as_user("put", f"/jobs/{new_job.id}", {"name": "new name"})
        assert st == 200 and body["job"]["startAt"] is None

    def test_update_running_job(self, as_user, new_running_job):
        st, _ = as_user("put", f"/jobs/{new_running_job.id}", {"startAt": iso(UTC() + timedelta(hours=5))})
        assert st == 422

    def test_update_not_owned_job(self, as_user, new_admin_job):
        assert as_user("put", f"/jobs/{new_admin_job.id}", {"name": "x"})[0] == 403

    def test_update_job_to_start_in_the_past(self, as_user, new_job):
        # fork: clamped to now (see test_create_job_in_the_past)
        st, _ = as_user("put", f"/jobs/{new_job.id}", {"startAt": iso(UTC() - timedelta(hours=5))})
        assert st == 200 and abs((Job.get(new_job.id).start_at - UTC()).total_seconds()) < 10

    def test_update_job_to_stop_before_start(self, as_user, new_job):
        st, _ = as_user("put", f"/jobs/{new_job.id}", {"startAt": iso(UTC() + timedelta(hours=5)),
                                                       "stopAt": iso(UTC() + timedelta(hours=1))})
        assert st == 422

    def test_delete_job(self, as_user, new_job_with_task):
        st, body = as_user("get", "/tasks", jobId=new_job_with_task.id)
        assert st == 200 and len(body["tasks"]) == 1
        assert as_user("delete", f"/jobs/{new_job_with_task.id}")[0] == 200
        assert as_user("get", "/tasks", jobId=new_job_with_task.id)[0] == 404  # tasks went by cascade

    def test_delete_not_owned_job(self, as_user, new_admin_job):
        assert as_user("delete", f"/jobs/{new_admin_job.id}")[0] == 403

    def test_get_tasks_from_job(self, as_user, new_job_with_task):
        st, body = as_user("get", "/tasks", jobId=new_job_with_task.id)
        assert st == 200 and len(body["tasks"]) == 1

    def test_get_tasks_from_not_owned_job(self, as_user, new_admin_job):
        assert as_user("get", "/tasks", jobId=new_admin_job.id)[0] == 403

    def test_add_task_to_job(self, as_user, new_job, new_task):
        st, body = as_user("put", f"/jobs/{new_job.id}/tasks/{new_task.id}")
        assert st == 200 and Task.get(new_task.id).job_id == new_job.id and body["job"]["id"] == new_job.id
        assert new_task.id in [t.id for t in Job.get(new_job.id).tasks]


# ================================================================= test_job_controller_superuser.py
class TestJobControllerSuperuser:
    def test_get_all_jobs(self, as_admin, new_job, new_admin_job):
        st, body = as_admin("get", "/jobs")
        assert st == 200 and len(body["jobs"]) == 2

    def test_update_not_owned_job(self, as_admin, new_job):
        st, body = as_admin("put", f"/jobs/{new_job.id}", {"name": "by admin",
                                                           "startAt": iso(UTC() + timedelta(hours=5))})
        assert st == 200 and Job.get(new_job.id).name == "by admin"

    def test_delete_not_owned_job(self, as_admin, new_job_with_task):
        assert as_admin("delete", f"/jobs/{new_job_with_task.id}")[0] == 200
        assert as_admin("get", "/tasks", jobId=new_job_with_task.id)[0] == 404

    def test_get_tasks_from_not_owned_job(self, as_admin, new_job_with_task):
        st, body = as_admin("get", "/tasks", jobId=new_job_with_task.id)
        assert st == 200 and len(body["tasks"]) == 1


# ================================================================= test_reservation_controller.py
def _reservation_body(user, start, end, rid=GPU):
    return {"title": "Test reservation", "description": "Test reservation", "resourceId": rid, "userId": user.id,
            "start": start, "end": end}


class TestReservationController:
    def test_create_reservation_unprivileged(self, as_user, new_user):
        _gpu()
        st, _ = as_user("post", "/reservations", _reservation_body(new_user, "2101-01-01T10:00:00.000Z",
                                                                   "2101-01-01T12:00:00.000Z"))
        assert st == 403  # no restriction covers the user

    def test_create_reservation(self, as_user, new_user, granted):
        _gpu()
        now = UTC()
        st, body = as_user("post", "/reservations", _reservation_body(new_user, iso(now + timedelta(hours=1)),
                                                                      iso(now + timedelta(hours=2))))
        assert st == 201 and Reservation.get(body["reservation"]["id"]) is not None

    def test_create_reservation_with_an_indefinite_restriction(self, as_user, new_user, restriction):
        restriction.starts_at = datetime.datetime(2101, 1, 1, 10)
        restriction.ends_at = None
        restriction.apply_to_user(new_user)
        restriction.apply_to_resource(_gpu())
        st, body = as_user("post", "/reservations", _reservation_body(new_user, "2101-01-02T10:00:00.000Z",
                                                                      "2101-01-02T12:00:00.000Z"))
        assert st == 201 and Reservation.get(body["reservation"]["id"]) is not None

    def test_create_reservation_starting_in_the_past(self, as_user, new_user, granted):
        # fork: reservations may start in the past (the reference commented its check out)
        _gpu()
        st, _ = as_user("post", "/reservations", _reservation_body(new_user, iso(UTC() - timedelta(hours=1)),
                                                                   iso(UTC() + timedelta(hours=1))))
        assert st == 201

    def test_create_reservation_with_permissions_just_for_a_part_of_it(self, as_user, new_user, restriction):
        restriction.starts_at = datetime.datetime(2101, 1, 1, 10)
        restriction.ends_at = datetime.datetime(2101, 1, 5, 10)
        restriction.apply_to_user(new_user)
        restriction.apply_to_resource(_gpu())
        st, _ = as_user("post", "/reservations", _reservation_body(new_user, "2101-01-04T10:00:00.000Z",
                                                                   "2101-01-06T12:00:00.000Z"))
        assert st == 403

    def test_create_reservation_outside_of_schedule(self, as_user, new_user, restriction):
        restriction.starts_at = datetime.datetime(2101, 1, 1, 10)
        restriction.ends_at = datetime.datetime(2101, 1, 5, 10)
        restriction.apply_to_user(new_user)
        s = RestrictionSchedule(schedule_days="1234567", hour_start=datetime.time(8), hour_end=datetime.time(10))
        s.save()
        restriction.add_schedule(s)
        restriction.apply_to_resource(_gpu())
        st, _ = as_user("post", "/reservations", _reservation_body(new_user, "2101-01-07T09:00:00.000Z",
                                                                   "2101-01-07T10:30:00.000Z"))
        assert st == 403

    def test_create_reservation_that_is_covered_by_two_separate_restrictions(self, as_user, new_user):
        r1 = Restriction(name="First", starts_at="2101-01-01T00:00:00.000Z", ends_at="2101-01-02T00:00:00.000Z",
                         is_global=False)
        r2 = Restriction(name="Second", starts_at="2101-01-02T00:00:00.000Z", ends_at="2101-01-02T23:59:00.000Z",
                         is_global=False)
        gpu = _gpu()
        for r in (r1, r2):
            r.apply_to_user(new_user)
            r.apply_to_resource(gpu)
        st, body = as_user("post", "/reservations", _reservation_body(new_user, "2101-01-01T10:00:00.000Z",
                                                                      "2101-01-02T12:00:00.000Z"))
        assert st == 201 and Reservation.get(body["reservation"]["id"]) is not None

    def test_update_reservation(self, as_user, future_reservation, granted):
        future_reservation.save()
        st, body = as_user("put", f"/reservations/{future_reservation.id}", {"title": "New title",
                                                                               "description": "New description"})
        assert st == 201 and body["reservation"]["title"] == "New title"
        assert Reservation.get(future_reservation.id).description == "New description"

    def test_update_reservation_unprivileged(self, as_user, future_reservation, new_admin):
        future_reservation.user_id = new_admin.id  # somebody else's
        future_reservation.save()
        assert as_user("put", f"/reservations/{future_reservation.id}", {"title": "New title"})[0] == 403

    def test_update_future_reservation_start(self, as_user, future_reservation, granted):
        future_reservation.save()
        new_start = future_reservation.start + timedelta(minutes=30)
        st, _ = as_user("put", f"/reservations/{future_reservation.id}", {"start": iso(new_start)})
        assert st == 201 and abs((Reservation.get(future_reservation.id).start - new_start).total_seconds()) < 1

    def test_update_active_reservation_start_forbidden(self, as_user, active_reservation, granted):
        active_reservation.save()
        st, _ = as_user("put", f"/reservations/{active_reservation.id}",
                        {"start": iso(active_reservation.start + timedelta(minutes=30))})
        assert st == 403

    def test_update_past_reservation_forbidden(self, as_user, past_reservation, granted):
        past_reservation.save()
        assert as_user("put", f"/reservations/{past_reservation.id}", {"title": "New title"})[0] == 403

    def test_delete_active_reservation_forbidden(self, as_user, active_reservation, granted):
        active_reservation.save()
        assert as_user("delete", f"/reservations/{active_reservation.id}")[0] == 403
        assert Reservation.get(active_reservation.id) is not None


# ================================================================= test_reservation_controller_superuser.py
class TestReservationControllerSuperuser:
    def test_after_updating_restriction_reservations_that_are_no_longer_valid_should_get_cancelled(
            self, as_admin, new_user, restriction, resource1):
        restriction.starts_at = UTC() - timedelta(hours=1)
        restriction.ends_at = UTC() + timedelta(days=2)
        restriction.apply_to_user(new_user)
        restriction.apply_to_resource(resource1)
        start = UTC() + timedelta(days=1)
        r = Reservation(user_id=new_user.id, title="t", description="d", resource_id=resource1.id, start=start,
                        end=start + timedelta(hours=2))
        r.save()
        st, _ = as_admin("put", f"/restrictions/{restriction.id}", {"endsAt": iso(UTC() + timedelta(hours=12))})
        assert st == 200
        db_session.remove()
        assert Reservation.get(r.id).is_cancelled
        # extending it again restores the reservation
        st, _ = as_admin("put", f"/restrictions/{restriction.id}", {"endsAt": iso(UTC() + timedelta(days=3))})
        assert st == 200
        db_session.remove()
        assert not Reservation.get(r.id).is_cancelled

    def test_update_past_reservation(self, as_admin, past_reservation, granted):
        past_reservation.save()
        st, body = as_admin("put", f"/reservations/{past_reservation.id}", {"title": "New title"})
        assert st == 201 and body["reservation"]["title"] == "New title"

    def test_create_reservation_starting_in_the_past(self, as_admin, new_admin, granted):
        _gpu()
        st, body = as_admin("post", "/reservations", _reservation_body(new_admin, iso(UTC() - timedelta(hours=2)),
                                                                       iso(UTC() + timedelta(hours=1))))
        assert st == 201 and Reservation.get(body["reservation"]["id"]) is not None

    def test_delete_active_reservation(self, as_admin, active_reservation, granted):
        active_reservation.save()
        assert as_admin("delete", f"/reservations/{active_reservation.id}")[0] == 200
        with pytest.raises(Exception):
            Reservation.get(active_reservation.id)


# ================================================================= test_restriction_controller.py
class TestRestrictionController:
    def test_get_all_restrictions_empty_response(self, as_user):
        st, body = as_user("get", "/restrictions")
        assert st == 200 and body == []

    def test_get_all_restrictions_with_data(self, as_user):
        Restriction(name="r", starts_at="2101-01-01T10:00:00.000Z", is_global=False).save()
        st, body = as_user("get", "/restrictions")
        assert st == 200 and len(body) == 1

    def test_get_user_restrictions(self, as_user, new_user, restriction):
        restriction.apply_to_user(new_user)
        st, body = as_user("get", "/restrictions", user_id=new_user.id)
        assert st == 200 and body[0]["id"] == restriction.id

    def test_get_users_group_restrictions(self, as_user, new_group_with_member, new_user, restriction):
        restriction.apply_to_group(new_group_with_member)
        st, body = as_user("get", "/restrictions", user_id=new_user.id, include_user_groups="true")
        assert st == 200 and [r["id"] for r in body] == [restriction.id]
        st, body = as_user("get", "/restrictions", user_id=new_user.id)
        assert st == 200 and body == []  # own restrictions only

    def test_get_group_restrictions(self, as_user, new_group, restriction):
        new_group.save()
        restriction.apply_to_group(new_group)
        st, body = as_user("get", "/restrictions", group_id=new_group.id)
        assert st == 200 and body[0]["id"] == restriction.id

    def test_get_resource_restrictions(self, as_user, resource1, restriction):
        restriction.apply_to_resource(resource1)
        st, body = as_user("get", "/restrictions", resource_id=resource1.id)
        assert st == 200 and body[0]["id"] == restriction.id

    def test_get_schedule_restrictions(self, as_user, active_schedule, restriction):
        restriction.add_schedule(active_schedule)
        st, body = as_user("get", "/restrictions", schedule_id=active_schedule.id)
        assert st == 200 and body[0]["id"] == restriction.id

    def test_create_restriction_unprivileged(self, as_user):
        st, _ = as_user("post", "/restrictions", {"name": "r", "startsAt": "2100-01-01T10:00:00.000Z",
                                                  "endsAt": "2101-02-01T10:00:00.000Z", "isGlobal": False})
        assert st == 403 and Restriction.query.count() == 0

    def test_update_restriction_unprivileged(self, as_user, restriction):
        restriction.save()
        assert as_user("put", f"/restrictions/{restriction.id}", {"name": "Modified"})[0] == 403
        assert Restriction.get(restriction.id).name == "TestRestriction"

    def test_apply_restriction_to_group_unprivileged(self, as_user, restriction, new_group):
        new_group.save()
        restriction.save()
        assert as_user("put", f"/restrictions/{restriction.id}/groups/{new_group.id}")[0] == 403
        assert new_group not in Restriction.get(restriction.id).groups

    def test_remove_resources_with_given_hostname_from_restriction(self, as_user, restriction, resource1):
        restriction.apply_to_resource(resource1)
        assert as_user("delete", f"/restrictions/{restriction.id}/hosts/{resource1.hostname}")[0] == 403
        assert resource1 in Restriction.get(restriction.id).resources

    def test_delete_restriction_unprivileged(self, as_user, restriction):
        restriction.save()
        assert as_user("delete", f"/restrictions/{restriction.id}")[0] == 403
        assert Restriction.get(restriction.id) is not None


# ================================================================= test_restriction_controller_superuser.py
class TestRestrictionControllerSuperuser:
    def test_create_restriction(self, as_admin):
        st, body = as_admin("post", "/restrictions", {"name": "r", "startsAt": "2100-01-01T10:00:00.000Z",
                                                      "endsAt": "2101-02-01T10:00:00.000Z", "isGlobal": False})
        assert st == 201 and Restriction.get(body["restriction"]["id"]) is not None

    def test_create_indefinte_retriction(self, as_admin):
        st, body = as_admin("post", "/restrictions", {"name": "r", "startsAt": "2100-01-01T10:00:00.000Z",
                                                      "isGlobal": False})
        assert st == 201 and Restriction.get(body["restriction"]["id"]).ends_at is None

    def test_create_restriction_missing_data(self, as_admin):
        st, _ = as_admin("post", "/restrictions", {"name": "r", "endsAt": "2101-02-01T10:00:00.000Z", "isGlobal": False})
        assert st == 400

    def test_update_restriction(self, as_admin, restriction):
        restriction.save()
        st, body = as_admin("put", f"/restrictions/{restriction.id}", {"name": "Modified name"})
        assert st == 200 and body["restriction"]["name"] == "Modified name"
        assert Restriction.get(restriction.id).name == "Modified name"

    def test_update_restriction_incorrect_data(self, as_admin, restriction):
        restriction.save()
        rid, old = restriction.id, (restriction.starts_at, restriction.ends_at)
        st, _ = as_admin("put", f"/restrictions/{rid}", {"startsAt": "2200-01-01T10:00:00.000Z",
                                                         "endsAt": "2199-02-01T10:00:00.000Z"})
        db_session.remove()
        r = Restriction.get(rid)
        assert st == 422 and (r.starts_at, r.ends_at) == old

    def test_update_nonexistent_restriction(self, as_admin):
        assert as_admin("put", "/restrictions/777", {"name": "Something"})[0] == 404

    def test_apply_restriction_to_group(self, as_admin, restriction, new_group):
        new_group.save()
        restriction.save()
        st, body = as_admin("put", f"/restrictions/{restriction.id}/groups/{new_group.id}")
        assert st == 200 and restriction in new_group.get_restrictions() and new_group in restriction.groups
        assert [g["id"] for g in body["restriction"]["groups"]] == [new_group.id]

    def test_apply_restriction_to_nonexistent_group(self, as_admin, restriction):
        restriction.save()
        assert as_admin("put", f"/restrictions/{restriction.id}/groups/777")[0] == 404

    def test_apply_nonexistent_restriction_to_group(self, as_admin, new_group):
        new_group.save()
        assert as_admin("put", f"/restrictions/777/groups/{new_group.id}")[0] == 404

    def test_apply_restriction_to_resource(self, as_admin, restriction, resource1):
        restriction.save()
        st, _ = as_admin("put", f"/restrictions/{restriction.id}/resources/{resource1.id}")
        assert st == 200 and restriction in resource1.get_restrictions() and resource1 in restriction.resources

    def test_apply_restriction_to_resources_by_hostname(self, as_admin, restriction, resource1):
        other = _gpu("GPU-" + "9" * 36, "node-a")
        elsewhere = _gpu("GPU-" + "8" * 36, "node-b")
        restriction.save()
        st, body = as_admin("put", f"/restrictions/{restriction.id}/hosts/node-a")
        assert st == 200
        got = set(Restriction.get(restriction.id).resources)
        assert {resource1, other} <= got and elsewhere not in got
        assert all(r.hostname == "node-a" for r in got)  # plus the daemon's 8 simulated node-a GPUs
        assert {resource1.id, other.id} <= {r["id"] for r in body["restriction"]["resources"]}

    def test_apply_restriction_to_resources_by_nonexistent_hostname(self, as_admin, restriction):
        restriction.save()
        assert as_admin("put", f"/restrictions/{restriction.id}/hosts/nonexistent")[0] == 404

    def test_apply_nonexistent_restriction_to_resources_by_hostname(self, as_admin, resource1):
        assert as_admin("put", f"/restrictions/777/hosts/{resource1.hostname}")[0] == 404

    def test_remove_resources_with_given_hostname_from_restriction(self, as_admin, restriction, resource1):
        other = _gpu("GPU-" + "8" * 36, "node-b")
        restriction.apply_to_resource(resource1)
        restriction.apply_to_resource(other)
        st, _ = as_admin("delete", f"/restrictions/{restriction.id}/hosts/{resource1.hostname}")
        assert st == 200 and Restriction.get(restriction.id).resources == [other]

    def test_remove_resources_with_nonexistent_hostname_from_restriction(self, as_admin, restriction):
        restriction.save()
        assert as_admin("delete", f"/restrictions/{restriction.id}/hosts/nonexistent")[0] == 404

    def test_remove_resources_with_given_hostname_from_nonexistent_restriction(self, as_admin, resource1):
        assert as_admin("delete", f"/restrictions/777/hosts/{resource1.hostname}")[0] == 404

    def test_apply_restriction_to_nonexistent_resource(self, as_admin, restriction):
        restriction.save()
        assert as_admin("put", f"/restrictions/{restriction.id}/resources/GPU-{'7' * 36}")[0] == 404

    def test_apply_nonexistent_restriction_to_resource(self, as_admin, resource1):
        assert as_admin("put", f"/restrictions/777/resources/{resource1.id}")[0] == 404

    def test_apply_restriction_to_schedule(self, as_admin, restriction, active_schedule):
        restriction.save()
        st, _ = as_admin("put", f"/restrictions/{restriction.id}/schedules/{active_schedule.id}")
        assert st == 200 and active_schedule in Restriction.get(restriction.id).schedules

    def test_apply_restriction_to_nonexistent_schedule(self, as_admin, restriction):
        restriction.save()
        assert as_admin("put", f"/restrictions/{restriction.id}/schedules/777")[0] == 404

    def test_apply_nonexistent_restriction_to_schedule(self, as_admin, active_schedule):
        assert as_admin("put", f"/restrictions/777/schedules/{active_schedule.id}")[0] == 404

    def test_apply_restriction_to_user(self, as_admin, restriction, new_user):
        restriction.save()
        st, _ = as_admin("put", f"/restrictions/{restriction.id}/users/{new_user.id}")
        assert st == 200 and restriction in new_user.get_restrictions() and new_user in restriction.users

    def test_apply_restriction_to_nonexistent_user(self, as_admin, restriction):
        restriction.save()
        assert as_admin("put", f"/restrictions/{restriction.id}/users/777")[0] == 404

    def test_apply_nonexistent_restriction_to_user(self, as_admin, new_user):
        assert as_admin("put", f"/restrictions/777/users/{new_user.id}")[0] == 404

    def test_delete_restriction(self, as_admin, restriction, new_user):
        restriction.apply_to_user(new_user)
        assert as_admin("delete", f"/restrictions/{restriction.id}")[0] == 200
        with pytest.raises(Exception):
            Restriction.get(restriction.id)
        assert User.get(new_user.id).get_restrictions() == []

    def test_delete_nonexistent_restriction(self, as_admin):
        assert as_admin("delete", "/restrictions/777")[0] == 404


# ================================================================= test_schedule_controller.py
class TestScheduleController:
    def test_create_schedule_unprivileged(self, as_user):
        st, _ = as_user("post", "/schedules", {"scheduleDays": ["Monday"], "hourStart": "8:00", "hourEnd": "16:00"})
        assert st == 403 and RestrictionSchedule.query.count() == 0

    def test_get_list_of_schedules(self, as_user, active_schedule):
        st, body = as_user("get", "/schedules")
        assert st == 200 and len(body) == 1

    def test_get_schedule_by_id(self, as_user, active_schedule):
        st, body = as_user("get", f"/schedules/{active_schedule.id}")
        assert st == 200 and body["schedule"]["id"] == active_schedule.id

    def test_get_nonexistent_schedule_by_id(self, as_user):
        assert as_user("get", "/schedules/777")[0] == 404

    def test_delete_schedule_unprivileged(self, as_user, active_schedule):
        assert as_user("delete", f"/schedules/{active_schedule.id}")[0] == 403
        assert RestrictionSchedule.get(active_schedule.id) is not None

    def test_update_schedule_unprivileged(self, as_user, active_schedule):
        st, _ = as_user("put", f"/schedules/{active_schedule.id}", {"scheduleDays": ["Monday"], "hourStart": "8:30",
                                                                    "hourEnd": "9:30"})
        assert st == 403 and RestrictionSchedule.get(active_schedule.id).hour_start == datetime.time(0, 0)


# ================================================================= test_schedule_controller_superuser.py
class TestScheduleControllerSuperuser:
    def test_create_schedule(self, as_admin):
        st, body = as_admin("post", "/schedules", {"scheduleDays": ["Monday", "Tuesday"], "hourStart": "8:00",
                                                   "hourEnd": "16:00"})
        assert st == 201 and RestrictionSchedule.get(body["schedule"]["id"]) is not None
        assert body["schedule"]["scheduleDays"] == ["Monday", "Tuesday"]

    def test_create_schedule_with_missing_start_hour(self, as_admin):
        assert as_admin("post", "/schedules", {"scheduleDays": ["Monday"], "hourEnd": "16:00"})[0] == 400

    def test_create_schedule_with_nonexistent_schedule_days(self, as_admin):
        st, _ = as_admin("post", "/schedules", {"scheduleDays": ["Mondayy"], "hourStart": "8:00", "hourEnd": "16:00"})
        assert st == 422

    def test_create_schedule_with_no_schedule_days(self, as_admin):
        assert as_admin("post", "/schedules", {"hourStart": "8:00", "hourEnd": "16:00"})[0] == 400

    def test_delete_schedule(self, as_admin, active_schedule):
        assert as_admin("delete", f"/schedules/{active_schedule.id}")[0] == 200
        with pytest.raises(Exception):
            RestrictionSchedule.get(active_schedule.id)

    def test_delete_nonexistent_schedule(self, as_admin):
        assert as_admin("delete", "/schedules/777")[0] == 404

    def test_update_schedule(self, as_admin, active_schedule):
        st, _ = as_admin("put", f"/schedules/{active_schedule.id}", {"scheduleDays": ["Monday"], "hourStart": "8:30",
                                                                     "hourEnd": "9:30"})
        s = RestrictionSchedule.get(active_schedule.id)
        assert st == 200 and s.hour_start == datetime.time(8, 30) and s.hour_end == datetime.time(9, 30)

    def test_update_nonexistent_schedule(self, as_admin):
        assert as_admin("put", "/schedules/777", {"hourStart": "8:30"})[0] == 404

    def test_get_list_of_schedules_superuser(self, as_admin):
        st, body = as_admin("get", "/schedules")
        assert st == 200 and body == []
        st, _ = as_admin("post", "/schedules", {"hourStart": "8:00", "hourEnd": "16:00", "scheduleDays": ["Monday"]})
        assert st == 201
        st, body = as_admin("get", "/schedules")
        assert st == 200 and len(body) == 1


# ================================================================= test_task_controller.py
_TASK_BODY = {"command": "python command.py", "hostname": "localhost",
              "cmdsegments": {"params": [{"name": "--batch_size", "value": "32"}, {"name": "--rank", "value": "2"}],
                              "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": "0"}]}}
_TASK_UPDATE = {"hostname": "remotehost", "command": "python command.py",
                "cmdsegments": {"params": [{"name": "--batch_size", "value": "64"}],
                                "envs": [{"name": "HIP_VISIBLE_DEVICES", "value": "1"}]}}


class TestTaskController:
    def test_create_task(self, as_user, new_job):
        st, body = as_user("post", f"/jobs/{new_job.id}/tasks", _TASK_BODY)
        assert st == 201 and body["task"]["command"] == "python command.py" and body["task"]["jobId"] == new_job.id
        assert len(Job.get(new_job.id).tasks) == 1 and Task.get(body["task"]["id"]).number_of_params == 2

    def test_delete_task(self, as_user, new_job, new_task):
        new_job.add_task(new_task)
        assert as_user("delete", f"/tasks/{new_task.id}")[0] == 200
        assert len(Task.all()) == 0 and len(Job.all()) == 1 and len(CommandSegment.all()) == 0

    def test_delete_not_owned_task(self, as_user, new_admin_job):
        task = new_admin_job.tasks[0]
        assert as_user("delete", f"/tasks/{task.id}")[0] == 403 and Task.get(task.id) is not None

    def test_update_task(self, as_user, new_job, new_task):
        new_job.add_task(new_task)
        st, body = as_user("put", f"/tasks/{new_task.id}", _TASK_UPDATE)
        t = Task.get(new_task.id)
        assert st == 201 and body["task"]["hostname"] == "remotehost"
        assert t.number_of_params == 1 and t.number_of_env_vars == 1

    def test_update_not_owned_task(self, as_user, new_admin_job):
        task = new_admin_job.tasks[0]
        assert as_user("put", f"/tasks/{task.id}", _TASK_UPDATE)[0] == 403
        assert Task.get(task.id).hostname == "node-a"


# ================================================================= test_task_controller_superuser.py
class TestTaskControllerSuperuser:
    def test_delete_not_owned_task(self, as_admin, new_job_with_task):
        task = new_job_with_task.tasks[0]
        assert as_admin("delete", f"/tasks/{task.id}")[0] == 200
        assert len(Task.all()) == 0 and len(Job.all()) == 1 and len(CommandSegment.all()) == 0

    def test_update_not_owned_task(self, as_admin, new_job_with_task):
        task = new_job_with_task.tasks[0]
        st, body = as_admin("put", f"/tasks/{task.id}", _TASK_UPDATE)
        t = Task.get(task.id)
        assert st == 201 and body["task"]["hostname"] == "remotehost"
        assert t.number_of_params == 1 and t.number_of_env_vars == 1


# ================================================================= test_user_controller{,_superuser}.py
class TestUserController:
    def test_user_signup_unprivileged(self, as_user):
        st, _ = as_user("post", "/user/create", {"username": "someone", "email": "a@b.org", "password": "password1"})
        assert st == 403 and User.query.filter_by(username="someone").count() == 0


class TestUserControllerSuperuser:
    _NEW = {"username": "newcomer", "email": "n@x.org", "password": "password1"}

    def test_on_signup_user_gets_added_to_a_default_group(self, as_admin):
        g = Group(name="defaults", is_default=True)
        g.save()
        st, body = as_admin("post", "/user/create", self._NEW)
        assert st == 201 and [x["name"] for x in body["user"]["groups"]] == ["defaults"]
        assert User.find_by_username("newcomer") in Group.get(g.id).users

    def test_on_signup_user_gets_added_to_all_default_groups_if_there_are_more_than_one(self, as_admin):
        for n in ("d1", "d2"):
            Group(name=n, is_default=True).save()
        Group(name="other").save()
        assert as_admin("post", "/user/create", self._NEW)[0] == 201
        assert {g.name for g in User.find_by_username("newcomer").groups} == {"d1", "d2"}

    def test_on_signup_user_does_not_belong_to_any_group_if_no_default_group_exists(self, as_admin):
        Group(name="other").save()
        assert as_admin("post", "/user/create", self._NEW)[0] == 201
        assert User.find_by_username("newcomer").groups == []
