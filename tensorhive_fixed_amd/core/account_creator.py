"""Interactive account creation (reference ``core/utils/AccountCreator.py:12-139``).

Prompts: username, email, password twice, admin?  New users join every default group.  On the
very first account it offers to create a default group ``users`` with a global, never-expiring
restriction (so that everybody can reserve every GPU until an admin narrows it).
"""
from __future__ import annotations

import click
from sqlalchemy.exc import IntegrityError

from ..database import db_session
from ..models.orm import Group, Restriction, Role, User
from ..utils import dates


class AccountCreator:
    def __init__(self):
        self.username = self.email = self.password = None
        self.is_admin = False

    def run_prompt(self) -> User | None:
        first = db_session.query(User).count() == 0
        self.username = click.prompt("[1/4] UNIX username", type=str)
        self.email = click.prompt("[2/4] email", type=str)
        while True:
            pw = click.prompt("[3/4] password", hide_input=True)
            pw2 = click.prompt("[3/4] repeat password", hide_input=True)
            if pw == pw2:
                self.password = pw
                break
            click.echo("Passwords do not match, try again")
        self.is_admin = click.confirm("[4/4] admin account?", default=first)
        user = self.create()
        if user is not None and first and not Group.get_default_groups():
            if click.confirm("Create a default group 'users' with a global permission (all GPUs, forever)?",
                             default=True):
                self.create_default_group(user)
        return user

    def create(self) -> User | None:
        roles = [Role(name="user")] + ([Role(name="admin")] if self.is_admin else [])
        try:
            user = User(username=self.username, email=self.email, password=self.password, roles=roles)
            user.save()
        except AssertionError as e:
            db_session.rollback()
            click.echo(f"Account not created: {e}")
            return None
        except IntegrityError:
            db_session.rollback()
            click.echo("Account not created: such user already exists")
            return None
        for g in Group.get_default_groups():
            g.add_user(user)
        click.echo(f"Account {user.username} created")
        return user

    @staticmethod
    def create_default_group(user: User) -> Group:
        g = Group(name="users", is_default=True)
        g.save()
        g.add_user(user)
        r = Restriction(name="Can always use everything", starts_at=dates.utcnow(), is_global=True)
        r.save()
        r.apply_to_group(g)
        return g
