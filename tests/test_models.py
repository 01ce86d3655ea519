"""ORM unit tests (reference ``tests/unit/models/*`` scenarios, plus the fork's fixes)."""
import datetime
from datetime import timedelta

import pytest
from sqlalchemy.exc import IntegrityError

from tensorhive_fixed_amd.database import db_session
from tensorhive_fixed_amd.models.orm import (CommandSegment, Group, Job, JobStatus, Reservation, Resource,
                                             Restriction, RestrictionSchedule, Role, SegmentType, Task,
                                             TaskStatus, User)
from tensorhive_fixed_amd.utils.exceptions import InvalidRequestException
from tensorhive_fixed_amd.utils.weekday import Weekday

NOW = datetime.datetime.utcnow


# ----------------------------------------------------------------------------- users / roles
def test_user_roles(new_user, new_admin):
    assert set(new_user.role_names) == {"user"}
    assert set(new_admin.role_names) == {"user", "admin"}
    assert new_admin.has_role("admin") and not new_user.has_role("admin")


@pytest.mark.parametrize("name", ["a", "a" * 31, "", "         ", "!@#$%^&*()[]{};<>?/", "nonurlfriendly!!!", "root"])
def test_invalid_usernames_rejected(tables, name):
    with pytest.raises(AssertionError):
        User(username=name, password="irrelevant").save()
    db_session.rollback()


def test_user_without_password_rejected(tables):
    with pytest.raises(IntegrityError):
        User(username="valid_username").save()
    db_session.rollback()


def test_duplicate_username_rejected(tables):
    User(username="valid_username", password="password1").save()
    with pytest.raises(IntegrityError):
        User(username="valid_username", password="password1").save()
    db_session.rollback()


def test_password_hash_verifies(new_user):
    assert new_user._hashed_password.startswith("$pbkdf2-sha256$")
    assert User.verify_hash("TEST PASSWORD", new_user._hashed_password)
    assert not User.verify_hash("wrong", new_user._hashed_password)


def test_user_reservations_exclude_cancelled(new_user, new_reservation):
    new_reservation.is_cancelled = True
    new_reservation.save()
    assert new_reservation not in new_user.get_reservations()
    assert new_reservation in new_user.get_reservations(include_cancelled=True)


def test_role_lookup(new_admin):
    assert {r.name for r in Role.find_by_user_id(new_admin.id)} == {"user", "admin"}


# ----------------------------------------------------------------------------- groups
def test_group_membership(new_user, new_group):
    new_group.save()
    new_group.add_user(new_user)
    assert new_user in new_group.users and new_group in new_user.groups
    with pytest.raises(InvalidRequestException):
        new_group.add_user(new_user)
    new_group.remove_user(new_user)
    assert new_user not in new_group.users
    with pytest.raises(InvalidRequestException):
        new_group.remove_user(new_user)


def test_default_groups(new_group):
    new_group.save()
    assert Group.get_default_groups() == []
    new_group.is_default = True
    new_group.save()
    other = Group(name="AnotherGroup", is_default=True)
    other.save()
    assert set(Group.get_default_groups()) == {new_group, other}
    assert Group.get(new_group.id).is_default


# ----------------------------------------------------------------------------- restrictions
def test_restriction_creation_and_validation(tables):
    start = NOW() + timedelta(minutes=5)
    r = Restriction(name="R", starts_at=start, ends_at=start + timedelta(hours=12))
    r.save()
    assert r.id is not None
    Restriction(name="Indefinite", starts_at=start).save()
    with pytest.raises(AssertionError):  # ends before it starts
        Restriction(name="bad", starts_at=NOW() + timedelta(hours=5), ends_at=NOW() + timedelta(minutes=1)).save()
    db_session.rollback()
    with pytest.raises(AssertionError):  # already expired
        Restriction(name="old", starts_at=NOW() - timedelta(hours=5), ends_at=NOW() - timedelta(hours=4)).save()
    db_session.rollback()


def test_restriction_string_dates(tables):
    r = Restriction(name="strings")
    r.starts_at = "2020-09-29T18:07:44.191Z"
    r.ends_at = "2120-09-30T18:07:44.191Z"
    r.save()
    assert r.ends_at.year == 2120


def test_global_restrictions(tables, resource1, resource2):
    start = NOW() + timedelta(minutes=5)
    g = Restriction(name="G", starts_at=start, ends_at=start + timedelta(hours=1), is_global=True)
    g.save()
    assert g in Restriction.get_global_restrictions()
    assert len(g.resources) == 0
    assert g in resource1.get_restrictions() and g in resource2.get_restrictions()
    assert g not in resource1.get_restrictions(include_global=False)


def test_restriction_assignment(restriction, new_user, new_group_with_member, new_user_2, resource1, inactive_schedule):
    restriction.apply_to_user(new_user_2)
    assert restriction in new_user_2.get_restrictions() and new_user_2 in restriction.users
    restriction.apply_to_group(new_group_with_member)
    assert restriction in new_group_with_member.get_restrictions()
    member = new_group_with_member.users[0]
    assert restriction in member.get_restrictions(include_group=True)
    assert restriction not in member.get_restrictions()
    assert set(restriction.get_all_affected_users()) == {new_user_2, member}
    restriction.apply_to_resource(resource1)
    assert restriction in resource1.get_restrictions(include_global=False)
    restriction.add_schedule(inactive_schedule)
    assert restriction in inactive_schedule.restrictions
    for fn, arg in ((restriction.apply_to_user, new_user_2), (restriction.apply_to_group, new_group_with_member),
                    (restriction.apply_to_resource, resource1), (restriction.add_schedule, inactive_schedule)):
        with pytest.raises(InvalidRequestException):
            fn(arg)


def test_restriction_removal_of_unassigned_fails(restriction, new_user, new_group, resource1, inactive_schedule):
    new_group.save()
    for fn, arg in ((restriction.remove_from_user, new_user), (restriction.remove_from_group, new_group),
                    (restriction.remove_from_resource, resource1), (restriction.remove_schedule, inactive_schedule)):
        with pytest.raises(InvalidRequestException):
            fn(arg)


def test_restriction_activity_by_dates(tables):
    active = Restriction(name="A", starts_at=NOW() - timedelta(hours=5), ends_at=NOW() + timedelta(hours=5))
    active.save()
    later = Restriction(name="B", starts_at=NOW() + timedelta(hours=1), ends_at=NOW() + timedelta(hours=5))
    later.save()
    assert active.is_active is True and later.is_active is False


def test_restriction_activity_by_schedules(tables, active_schedule, inactive_schedule):
    r = Restriction(name="A", starts_at=NOW() - timedelta(hours=5), ends_at=NOW() + timedelta(hours=5))
    r.save()
    r.add_schedule(inactive_schedule)
    assert r.is_active is False
    r.add_schedule(active_schedule)
    assert r.is_active is True


# ----------------------------------------------------------------------------- schedules
def test_schedule_expressions(tables):
    RestrictionSchedule(schedule_days="12345", hour_start=datetime.time(8), hour_end=datetime.time(15)).save()
    s = RestrictionSchedule(schedule_days="1458", hour_start=datetime.time(8), hour_end=datetime.time(15))
    with pytest.raises(AssertionError):
        s.save()
    db_session.rollback()
    s = RestrictionSchedule(schedule_days="1123", hour_start=datetime.time(8), hour_end=datetime.time(15))
    with pytest.raises(AssertionError):
        s.save()
    db_session.rollback()
    s = RestrictionSchedule(schedule_days=[Weekday.Monday, Weekday.Tuesday], hour_start=datetime.time(8),
                            hour_end=datetime.time(15))
    s.save()
    d = s.as_dict()
    assert s.schedule_days == "12" and d["scheduleDays"] == ["Monday", "Tuesday"] and d["hourStart"] == "08:00"


def test_schedule_is_active_today_only(tables):
    today = str(NOW().weekday() + 1)
    on = RestrictionSchedule(schedule_days=today, hour_start=datetime.time(0), hour_end=datetime.time(23, 59, 59))
    on.save()
    off = RestrictionSchedule(schedule_days="1234567".replace(today, ""), hour_start=datetime.time(0),
                              hour_end=datetime.time(23, 59, 59))
    off.save()
    assert on.is_active is True and off.is_active is False


# ----------------------------------------------------------------------------- resources
def test_resource_lookup(resource1, resource2):
    assert Resource.get_by_name("Custom name") == [resource2] or Resource.get_by_name("Custom name") == resource2
    assert resource1 in Resource.get_by_hostname("node-a")


# ----------------------------------------------------------------------------- reservations
def test_reservation_overlaps(new_reservation, new_reservation_2):
    new_reservation.save()
    off = timedelta(minutes=5)
    for a, b in ((off, -off), (-off, -off), (off, off), (-off, off)):
        new_reservation_2.start = new_reservation.start + a
        new_reservation_2.end = new_reservation.end + b
        with pytest.raises(AssertionError):
            new_reservation_2.save()
        db_session.rollback()


def test_cancelled_reservation_does_not_block(new_reservation, new_reservation_2):
    new_reservation.is_cancelled = True
    new_reservation.save()
    off = timedelta(minutes=5)
    for a, b in ((off, -off), (-off, -off), (off, off), (-off, off)):
        new_reservation_2.start = new_reservation.start + a
        new_reservation_2.end = new_reservation.end + b
        new_reservation_2.save()


def test_reservation_time_format(new_reservation):
    start = NOW() + timedelta(hours=3)
    end = start + timedelta(minutes=400)
    with pytest.raises(ValueError):
        new_reservation.start = start.strftime("%Y_%m_%dT%H:%M:%S.%fZ")
    new_reservation.start = start.strftime("%Y-%m-%dT%H:%M:%S.%fZ")
    new_reservation.end = end.strftime("%Y-%m-%dT%H:%M:%S.%fZ")
    new_reservation.save()


@pytest.mark.parametrize("start,dur", [(timedelta(hours=10), timedelta(hours=-20)),
                                       (timedelta(hours=1), timedelta(minutes=29, seconds=59)),
                                       (timedelta(hours=1), timedelta(days=8, seconds=1))])
def test_reservation_duration_limits(new_reservation, start, dur):
    new_reservation.start = NOW() + start
    new_reservation.end = new_reservation.start + dur
    with pytest.raises(AssertionError):
        new_reservation.save()
    db_session.rollback()


def test_current_events_skip_cancelled(new_reservation, new_reservation_2):
    new_reservation.start = NOW() - timedelta(minutes=10)
    new_reservation.end = NOW() + timedelta(minutes=60)
    new_reservation.save()
    assert new_reservation in Reservation.current_events()
    new_reservation.is_cancelled = True
    new_reservation.save()
    new_reservation_2.save()
    cur = Reservation.current_events()
    assert new_reservation not in cur and new_reservation_2 in cur


def test_upcoming_events(future_reservation, resource1):
    future_reservation.save()
    assert Reservation.upcoming_events_for_resource(resource1.id, timedelta(hours=6)) == [future_reservation]
    assert Reservation.upcoming_events_for_resource(resource1.id, timedelta(hours=1)) == []


def test_reservation_json_dates(new_reservation):
    new_reservation.save()
    d = new_reservation.as_dict()
    assert d["start"].endswith("+00:00") and d["userName"] == "administrantee"
    assert set(d) >= {"id", "title", "resourceId", "userId", "start", "end", "isCancelled"}


# ----------------------------------------------------------------------------- jobs / tasks
def test_job_task_membership(new_job, new_task):
    new_job.add_task(new_task)
    assert new_task in new_job.tasks and new_task.job is new_job
    with pytest.raises(InvalidRequestException):
        new_job.add_task(new_task)
    new_job.remove_task(new_task)
    assert new_task not in new_job.tasks
    with pytest.raises(InvalidRequestException):
        new_job.remove_task(new_task)


def test_job_status_follows_tasks(new_job_with_task, new_task_2):
    job = new_job_with_task
    t = job.tasks[0]
    t.status = TaskStatus.unsynchronized
    assert job.status is JobStatus.unsynchronized
    t.status = TaskStatus.running
    assert job.status is JobStatus.running
    new_task_2.status = TaskStatus.not_running
    job.add_task(new_task_2)
    assert job.status is JobStatus.running
    t.status = TaskStatus.terminated
    assert job.status is JobStatus.terminated
    t.status = TaskStatus.not_running
    assert job.status is JobStatus.not_running


def test_job_queue(new_job_with_task):
    job = new_job_with_task
    job.enqueue()
    assert job.status is JobStatus.pending and job in Job.get_job_queue()
    with pytest.raises(AssertionError):
        job.enqueue()
    job.tasks[0].status = TaskStatus.running
    assert job.status is JobStatus.running and job in Job.get_jobs_running_from_queue()
    assert job not in Job.get_job_queue()
    job.tasks[0].status = TaskStatus.terminated
    assert job.is_queued is False  # leaving `running` unqueues it (it is not rescheduled)
    assert job not in Job.get_job_queue()


def test_job_dequeue(new_job_with_task):
    with pytest.raises(AssertionError):
        new_job_with_task.dequeue()
    new_job_with_task.enqueue()
    new_job_with_task.dequeue()
    assert new_job_with_task.status is JobStatus.not_running and not new_job_with_task.is_queued


def test_job_times(new_job):
    new_job.start_at = NOW() - timedelta(hours=1)  # past start -> now (fork behaviour)
    assert abs((new_job.start_at - NOW()).total_seconds()) < 5
    new_job.stop_at = NOW() - timedelta(hours=2)
    with pytest.raises(AssertionError):
        new_job.save()
    db_session.rollback()


def test_task_full_command(tables):
    t = Task(command="python train.py", hostname="node-a")
    t.save()
    t.add_cmd_segment(CommandSegment(name="HIP_VISIBLE_DEVICES", segment_type=SegmentType.env_variable), "0,1")
    t.add_cmd_segment(CommandSegment(name="--lr", segment_type=SegmentType.parameter), "0.1")
    t.add_cmd_segment(CommandSegment(name="--nproc_per_node=", segment_type=SegmentType.parameter), "2")
    t.add_cmd_segment(CommandSegment(name="-v", segment_type=SegmentType.parameter), "")
    assert t.full_command == "HIP_VISIBLE_DEVICES=0,1 python train.py --lr 0.1 --nproc_per_node=2 -v"
    assert t.number_of_params == 3 and t.number_of_env_vars == 1
    assert t.as_dict()["fullCommand"] == t.full_command


def test_task_segment_removal_reindexes(tables):
    t = Task(command="run", hostname="node-a")
    t.save()
    segs = [CommandSegment(name=f"--p{i}", segment_type=SegmentType.parameter) for i in range(3)]
    for i, s in enumerate(segs):
        t.add_cmd_segment(s, str(i))
    t.remove_cmd_segment(segs[0])
    assert t.full_command == "run --p1 1 --p2 2"
    assert sorted(lk.index for lk in t.segment_links) == [1, 2]
    with pytest.raises(Exception):
        t.remove_cmd_segment(segs[0])


# ----------------------------------------------------------------------------- infrastructure filter
def test_filter_infrastructure_by_restrictions(new_user, resource1, resource2):
    infra = {"node-a": {"GPU": {resource1.id: {"name": "x"}}, "CPU": {}},
             "node-b": {"GPU": {resource2.id: {"name": "y"}}, "CPU": {}}}
    import copy

    assert new_user.filter_infrastructure_by_user_restrictions(copy.deepcopy(infra)) == {}  # GPU-less hosts dropped
    r = Restriction(name="one", starts_at=NOW() - timedelta(hours=1))
    r.save()
    r.apply_to_resource(resource1)
    r.apply_to_user(new_user)
    out = new_user.filter_infrastructure_by_user_restrictions(copy.deepcopy(infra))
    assert list(out["node-a"]["GPU"]) == [resource1.id]
    assert "node-b" not in out
    g = Restriction(name="global", starts_at=NOW() - timedelta(hours=1), is_global=True)
    g.save()
    g.apply_to_user(new_user)
    out = new_user.filter_infrastructure_by_user_restrictions(copy.deepcopy(infra))
    assert list(out["node-b"]["GPU"]) == [resource2.id]
