"""Empty stand-in for ``opengen`` (0.7.1, requirements.txt:21).  TEST TOOLING ONLY: the
reference's solver.py imports it at module level; the golden generator only uses
``Solver.create_x_init`` (solver.py:103-136), which never touches opengen."""
