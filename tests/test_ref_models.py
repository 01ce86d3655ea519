"""Scenario-for-scenario counterparts of the reference model tests (``tests/unit/models/test_*.py``,
56 functions counting each parametrised case of ``test_exception_on_creating_user_with_invalid_username``
once, as the reference file does).  One class per reference module, methods named as there."""
import datetime
from datetime import timedelta

import pytest
from click.testing import CliRunner
from sqlalchemy.exc import IntegrityError

from tensorhive_fixed_amd.database import db_session
from tensorhive_fixed_amd.models.orm import (Group, Job, JobStatus, Reservation, Resource, Restriction,
                                             RestrictionSchedule, TaskStatus, User)
from tensorhive_fixed_amd.utils.exceptions import InvalidRequestException
from tensorhive_fixed_amd.utils.weekday import Weekday

NOW = datetime.datetime.utcnow


# ================================================================= test_account_creator.py
class TestAccountCreator:
    @pytest.mark.parametrize("test_name, test_input", [
        ("will_pass", ["some_username", "some@email.com", "some_password", "some_password", "y", "n"])])
    def test_prompts(self, tables, test_name, test_input):
        import click

        from tensorhive_fixed_amd.core.account_creator import AccountCreator

        @click.command()
        def wrapper():
            assert AccountCreator().run_prompt() is not None

        r = CliRunner().invoke(wrapper, input="\n".join(test_input) + "\n")
        assert r.exception is None, r.output
        u = User.find_by_username("some_username")
        assert set(u.role_names) == {"user", "admin"} and Group.get_default_groups() == []


# ================================================================= test_group_model.py
class TestGroupModel:
    def test_group_creation(self, tables):
        assert Group(name="test").save().id is not None

    def test_adding_user_to_a_group(self, new_user, new_group):
        new_group.save()
        new_group.add_user(new_user)
        assert new_user in new_group.users and new_group in new_user.groups

    def test_removing_user_from_a_group(self, new_group_with_member):
        user = new_group_with_member.users[0]
        new_group_with_member.remove_user(user)
        assert user not in new_group_with_member.users and new_group_with_member not in user.groups

    def test_removing_user_from_a_group_that_he_doesnt_belong_to_fails(self, new_user, new_group):
        new_group.save()
        with pytest.raises(InvalidRequestException):
            new_group.remove_user(new_user)

    def test_adding_user_to_a_group_that_he_is_already_in_fails(self, new_group_with_member):
        with pytest.raises(InvalidRequestException):
            new_group_with_member.add_user(new_group_with_member.users[0])

    def test_marking_group_as_a_default(self, new_group):
        new_group.is_default = True
        new_group.save()
        assert Group.get(new_group.id).is_default and new_group in Group.get_default_groups()

    def test_get_default_group(self, new_group):
        new_group.is_default = True
        new_group.save()
        assert new_group in Group.get_default_groups()

    def test_get_default_without_default_group(self, new_group):
        new_group.save()
        assert len(Group.get_default_groups()) == 0

    def test_more_than_one_default_group(self, new_group):
        new_group.is_default = True
        new_group.save()
        another = Group(name="AnotherGroup", is_default=True)
        another.save()
        defaults = Group.get_default_groups()
        assert new_group in defaults and another in defaults


# ================================================================= test_job_model.py
class TestJobModel:
    def test_job_creation(self, new_user):
        assert Job(name="job_name", description="testDescription", user_id=new_user.id).save().id is not None

    def test_adding_task_to_a_job(self, new_task, new_job):
        new_job.add_task(new_task)
        assert new_task in new_job.tasks and new_job is new_task.job

    def test_removing_task_from_a_job(self, new_job_with_task):
        task = new_job_with_task.tasks[0]
        new_job_with_task.remove_task(task)
        assert task not in new_job_with_task.tasks and new_job_with_task is not task.job

    def test_removing_task_from_a_job_that_he_doesnt_belong_to_fails(self, new_task, new_job):
        with pytest.raises(InvalidRequestException):
            new_job.remove_task(new_task)

    def test_adding_task_to_a_job_that_he_is_already_in_fails(self, new_job_with_task):
        with pytest.raises(InvalidRequestException):
            new_job_with_task.add_task(new_job_with_task.tasks[0])

    def test_synchronizing_job(self, new_job_with_task, new_task_2):
        job = new_job_with_task
        job._status = JobStatus.unsynchronized
        task = job.tasks[0]
        task.status = TaskStatus.unsynchronized
        assert job.status is JobStatus.unsynchronized
        task.status = TaskStatus.running
        assert job.status is JobStatus.running
        new_task_2.status = TaskStatus.not_running
        job.add_task(new_task_2)
        assert job.status is JobStatus.running
        task.status = TaskStatus.terminated
        assert job.status is JobStatus.terminated
        task.status = TaskStatus.not_running
        assert job.status is JobStatus.not_running


# ================================================================= test_reservation_model.py
class TestReservationModel:
    def test_reservation_creation(self, new_reservation):
        new_reservation.save()
        assert Reservation.get(new_reservation.id) is new_reservation

    def test_interfering_reservation_cannot_be_saved(self, new_reservation, new_reservation_2):
        new_reservation.save()
        off = timedelta(minutes=5)
        # | A  A |,  A | A |,  | A | A,  A | | A
        for a, b in ((off, -off), (-off, -off), (off, off), (-off, off)):
            new_reservation_2.start = new_reservation.start + a
            new_reservation_2.end = new_reservation.end + b
            with pytest.raises(AssertionError):
                new_reservation_2.save()
            db_session.rollback()

    def test_cancelled_reservation_does_not_cause_interference_with_others(self, new_reservation, new_reservation_2):
        new_reservation.is_cancelled = True
        new_reservation.save()
        off = timedelta(minutes=5)
        for a, b in ((off, -off), (-off, -off), (off, off), (-off, off)):
            new_reservation_2.start = new_reservation.start + a
            new_reservation_2.end = new_reservation.end + b
            new_reservation_2.save()
        assert Reservation.get(new_reservation_2.id) is not None

    def test_string_time_format_conversion(self, new_reservation):
        start = NOW() + timedelta(hours=3)
        end = start + timedelta(minutes=400)
        with pytest.raises(ValueError):
            new_reservation.start = start.strftime("%Y_%m_%dT%H:%M:%S.%fZ")
        new_reservation.start = start.strftime("%Y-%m-%dT%H:%M:%S.%fZ")
        new_reservation.end = end.strftime("%Y-%m-%dT%H:%M:%S.%fZ")
        new_reservation.save()
        assert abs((Reservation.get(new_reservation.id).start - start).total_seconds()) < 1e-3

    def test_invalid_reservation_time_range(self, new_reservation):
        # end before start, shorter than 30 minutes, longer than 8 days
        for a, d in ((timedelta(hours=10), timedelta(hours=-20)), (timedelta(hours=1), timedelta(minutes=29)),
                     (timedelta(hours=1), timedelta(days=8, minutes=1))):
            new_reservation.start = NOW() + a
            new_reservation.end = new_reservation.start + d
            with pytest.raises(AssertionError):
                new_reservation.save()
            db_session.rollback()

    def test_current_events_will_only_return_non_cancelled_reservations(self, new_reservation, new_reservation_2):
        new_reservation.start = NOW() - timedelta(minutes=10)
        new_reservation.end = NOW() + timedelta(minutes=60)
        new_reservation.save()
        assert new_reservation in Reservation.current_events()
        new_reservation.is_cancelled = True
        new_reservation.save()
        new_reservation_2.save()
        cur = Reservation.current_events()
        assert new_reservation not in cur and new_reservation_2 in cur


# ================================================================= test_resource_model.py
class TestResourceModel:
    def test_resource_creation(self, tables):
        r = Resource(id="GPU-34943e60-0acd-4c31-b96e-02f88cc156f3")
        r.save()
        assert Resource.get(r.id) is not None


# ================================================================= test_restriction_model.py
class TestRestrictionModel:
    def test_restriction_creation(self, tables):
        s = NOW() + timedelta(minutes=5)
        r = Restriction(name="TestRestriction", starts_at=s, ends_at=s + timedelta(hours=12), is_global=False)
        r.save()
        assert r.id is not None

    def test_indefinite_restriction_creation(self, tables):
        r = Restriction(name="TestRestriction", starts_at=NOW() + timedelta(minutes=5), is_global=False)
        r.save()
        assert r.id is not None and r.ends_at is None

    def test_get_global_restrictions_returns_them(self, tables):
        s = NOW() + timedelta(minutes=5)
        r = Restriction(name="TestRestriction", starts_at=s, ends_at=s + timedelta(hours=12), is_global=True)
        r.save()
        assert r in Restriction.get_global_restrictions()

    def test_apply_restriction_to_user(self, restriction, new_user):
        restriction.apply_to_user(new_user)
        assert restriction in new_user.get_restrictions() and new_user in restriction.users

    def test_apply_restriction_to_group(self, restriction, new_group):
        new_group.save()
        restriction.apply_to_group(new_group)
        assert restriction in new_group.get_restrictions() and new_group in restriction.groups

    def test_group_restrictions_apply_to_its_members(self, restriction, new_group_with_member):
        restriction.apply_to_group(new_group_with_member)
        assert restriction in new_group_with_member.get_restrictions()
        assert restriction in new_group_with_member.users[0].get_restrictions(include_group=True)
        assert new_group_with_member in restriction.groups

    def test_it_should_be_impossible_to_create_restriction_with_end_time_happening_before_start_time(self, tables):
        r = Restriction(name="Test", starts_at=NOW() + timedelta(hours=5), ends_at=NOW() + timedelta(minutes=1),
                        is_global=False)
        with pytest.raises(AssertionError):
            r.save()

    def test_it_should_be_impossible_to_create_or_edit_restriction_that_already_expired(self, tables):
        s = NOW() - timedelta(hours=5)
        r = Restriction(name="Test", starts_at=s, ends_at=s + timedelta(hours=1), is_global=False)
        with pytest.raises(AssertionError):
            r.save()

    def test_apply_restriction_to_resource(self, restriction, resource1):
        restriction.apply_to_resource(resource1)
        assert restriction in resource1.get_restrictions(include_global=False) and resource1 in restriction.resources

    def test_global_restriction_applies_to_all_resources(self, restriction, resource1, resource2):
        restriction.is_global = True
        restriction.save()
        assert len(restriction.resources) == 0
        assert restriction in resource1.get_restrictions() and restriction in resource2.get_restrictions()

    def test_restriction_without_schedules_is_active_only_when_between_start_and_end_dates(self, tables):
        active = Restriction(name="A", starts_at=NOW() - timedelta(hours=5), ends_at=NOW() + timedelta(hours=5),
                             is_global=False)
        active.save()
        inactive = Restriction(name="I", starts_at=NOW() + timedelta(hours=1), ends_at=NOW() + timedelta(hours=5),
                               is_global=False)
        inactive.save()
        assert active.is_active is True and inactive.is_active is False

    def test_restriction_with_schedules_is_active_only_when_at_least_one_of_its_schedules_is_active(
            self, active_schedule, inactive_schedule):
        r = Restriction(name="A", starts_at=NOW() - timedelta(hours=5), ends_at=NOW() + timedelta(hours=5),
                        is_global=False)
        r.save()
        r.add_schedule(inactive_schedule)
        assert r.is_active is False
        r.add_schedule(active_schedule)
        assert r.is_active is True

    def test_restriction_with_dates_passed_as_string_gets_added_successfully(self, tables):
        r = Restriction(name="Test", starts_at="2100-01-01T10:00:00.000Z", ends_at="2101-01-01T10:00:00.000Z",
                        is_global=False)
        r.save()
        assert Restriction.get(r.id).starts_at == datetime.datetime(2100, 1, 1, 10)

    def test_when_trying_to_apply_restriction_to_the_same_group_twice_an_exception_is_thrown(self, restriction,
                                                                                            new_group):
        new_group.save()
        restriction.apply_to_group(new_group)
        with pytest.raises(InvalidRequestException):
            restriction.apply_to_group(new_group)

    def test_when_trying_to_apply_restriction_to_the_same_user_twice_an_exception_is_thrown(self, restriction,
                                                                                           new_user):
        restriction.apply_to_user(new_user)
        with pytest.raises(InvalidRequestException):
            restriction.apply_to_user(new_user)

    def test_when_trying_to_add_an_already_assigned_schedule_to_restriction_an_exception_is_thrown(
            self, restriction, inactive_schedule):
        restriction.add_schedule(inactive_schedule)
        with pytest.raises(InvalidRequestException):
            restriction.add_schedule(inactive_schedule)

    def test_when_trying_to_add_an_already_assigned_resource_to_restriction_an_exception_is_thrown(
            self, restriction, resource1):
        restriction.apply_to_resource(resource1)
        with pytest.raises(InvalidRequestException):
            restriction.apply_to_resource(resource1)

    def test_when_trying_to_remove_restriction_from_group_that_wasnt_assigned_to_it_an_exception_is_thrown(
            self, restriction, new_group):
        new_group.save()
        with pytest.raises(InvalidRequestException):
            restriction.remove_from_group(new_group)

    def test_when_trying_to_remove_restriction_from_user_that_wasnt_assigned_to_it_an_exception_is_thrown(
            self, restriction, new_user):
        with pytest.raises(InvalidRequestException):
            restriction.remove_from_user(new_user)

    def test_when_trying_to_remove_schedule_that_wasnt_assigned_to_restriction_an_exception_is_thrown(
            self, restriction, inactive_schedule):
        with pytest.raises(InvalidRequestException):
            restriction.remove_schedule(inactive_schedule)

    def test_when_trying_to_remove_restriction_from_resource_that_wasnt_assigned_to_it_an_exception_is_thrown(
            self, restriction, resource1):
        with pytest.raises(InvalidRequestException):
            restriction.remove_from_resource(resource1)

    def test_get_all_affected_users_will_return_all_users_affected_by_given_restriction(
            self, restriction, new_user_2, new_group_with_member):
        restriction.apply_to_group(new_group_with_member)
        restriction.apply_to_user(new_user_2)
        member = new_group_with_member.users[0]
        assert new_user_2 in restriction.users and member not in restriction.users
        affected = restriction.get_all_affected_users()
        assert new_user_2 in affected and member in affected


# ================================================================= test_restrictionschedule_model.py
class TestRestrictionscheduleModel:
    def test_schedule_creation(self, tables):
        s = RestrictionSchedule(schedule_days="12345", hour_start=datetime.time(8), hour_end=datetime.time(15))
        s.save()
        assert s.id is not None

    def test_cannot_create_schedule_with_wrong_schedule_expression(self, tables):
        for days in ("1458", "0", "12a"):
            s = RestrictionSchedule(schedule_days=days, hour_start=datetime.time(8), hour_end=datetime.time(15))
            with pytest.raises(AssertionError):
                s.save()
            db_session.rollback()

    def test_add_schedule_to_restriction(self, restriction, active_schedule):
        restriction.add_schedule(active_schedule)
        assert active_schedule in restriction.schedules and restriction in active_schedule.restrictions

    def test_schedule_is_active_method_returns_valid_status(self, tables):
        today = str(NOW().weekday() + 1)
        a = RestrictionSchedule(schedule_days=today, hour_start=datetime.time(0), hour_end=datetime.time(23, 59, 59))
        a.save()
        i = RestrictionSchedule(schedule_days="1234567".replace(today, ""), hour_start=datetime.time(0),
                                hour_end=datetime.time(23, 59, 59))
        i.save()
        assert a.is_active is True and i.is_active is False

    def test_schedule_with_schedule_days_as_list_of_enums_gets_saved_successfully(self, tables):
        s = RestrictionSchedule(schedule_days=[Weekday.Monday, Weekday.Tuesday], hour_start=datetime.time(8),
                                hour_end=datetime.time(15))
        s.save()
        assert RestrictionSchedule.get(s.id).schedule_days == "12"


# ================================================================= test_user_model.py
class TestUserModel:
    def test_user_creation(self, new_user, new_admin):
        assert new_user.id and set(new_user.role_names) == {"user"}
        assert new_admin.id and set(new_admin.role_names) == {"admin", "user"}

    @pytest.mark.parametrize("test_name, test_username", [
        ("too_short", "a"), ("too_long", "a" * 31), ("empty", ""), ("sneaky", "         "),
        ("special", "!@#$%^&*()[]{};<>?/"), ("blacklisted", "nonurlfriendly!!!"), ("blacklisted", "jerk")])
    def test_exception_on_creating_user_with_invalid_username(self, tables, test_name, test_username):
        with pytest.raises(AssertionError):
            User(username=test_username, password="irrelevant_password").save()
        db_session.rollback()

    def test_exception_on_creating_user_with_no_password(self, tables):
        with pytest.raises((IntegrityError, AssertionError)):
            User(username="valid_username").save()
        db_session.rollback()

    def test_exception_on_creating_user_with_not_unique_username(self, tables):
        with pytest.raises(IntegrityError):
            User(username="valid_username", password="irrelevant_password").save()
            User(username="valid_username", password="irrelevant_password").save()
        db_session.rollback()

    def test_get_users_reservations(self, new_user, new_reservation):
        new_reservation.save()
        assert new_reservation in new_user.get_reservations()

    def test_get_users_reservations_does_not_include_cancelled_reservations_by_default(self, new_user,
                                                                                       new_reservation):
        new_reservation.is_cancelled = True
        new_reservation.save()
        assert new_reservation not in new_user.get_reservations()
        assert new_reservation in new_user.get_reservations(include_cancelled=True)
