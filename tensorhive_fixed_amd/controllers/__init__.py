"""REST controllers (business functions separated from transport; reference ``controllers/*.py``).

Every public function here is bound to one operation of :mod:`..api.spec`; it receives the
validated path/query parameters and body and returns ``(content, status)``.  Business functions
(``business_execute``, ``business_stop``, ``business_spawn``, ...) take no request context so the
job-scheduling service can call them directly.
"""
