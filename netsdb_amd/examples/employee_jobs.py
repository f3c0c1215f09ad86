"""A UDF library as a remote client registers it (reference: sharedLibraries like
SillySelection / SimpleAggregation compiled into .so files and sent with registerType)."""
from netsdb_amd.computations import AggregateComp, ScanSet, SelectionComp, WriteSet
from netsdb_amd.lambdas import make_lambda_from_member, make_lambda_from_self
from netsdb_amd.objects.builtin import DepartmentTotal, Employee
from netsdb_amd.objects.record import RecordBatch


class OlderThan(SelectionComp):
    def __init__(self, age):
        super().__init__()
        self.age = age

    def get_selection(self, e):
        return make_lambda_from_member(e, "age") > self.age

    def get_projection(self, e):
        return make_lambda_from_self(e)


class SalaryByDept(AggregateComp):
    def get_key_projection(self, e):
        return make_lambda_from_member(e, "department")

    def get_value_projection(self, e):
        return make_lambda_from_member(e, "salary")

    def make_output(self, keys, values):
        return RecordBatch.from_objects([DepartmentTotal(k, float(v)) for k, v in zip(keys, values.tolist())],
                                        DepartmentTotal)


def select_older(client, db, src, dst, age):
    client.create_set(db, dst, Employee)
    stats = client.execute_computations(WriteSet(db, dst).set_input(OlderThan(age).set_input(ScanSet(db, src, Employee))))
    return {"seconds": stats["seconds"]}


def totals(client, db, src, dst):
    client.create_set(db, dst, DepartmentTotal)
    client.execute_computations(WriteSet(db, dst).set_input(SalaryByDept().set_input(ScanSet(db, src, Employee))))
    return True


def plan(client, db, src, age):
    return WriteSet(db, "x").set_input(OlderThan(age).set_input(ScanSet(db, src, Employee)))


JOBS = {"select_older": select_older, "totals": totals, "plan": plan}


# --------------------------------------------------------------------------- a UDF library for remote graphs
# (computation classes + record types a remote client references BY NAME in a declarative graph, after
# register_type("netsdb_amd.examples.employee_jobs"); the server imports only allow-listed modules)
from netsdb_amd.computations import JoinComp  # noqa: E402
from netsdb_amd.lambdas import make_lambda  # noqa: E402
from netsdb_amd.objects.record import PDBObject  # noqa: E402


class Department(PDBObject):
    name: str
    floor: int


class EmpFloor(PDBObject):
    name: str
    department: str
    floor: int
    salary: float


class EmpJoinDepartment(JoinComp):
    """Employee.department == Department.name -> EmpFloor."""

    def get_selection(self, e, d):
        return make_lambda_from_member(e, "department") == make_lambda_from_member(d, "name")

    def get_projection(self, e, d):
        return make_lambda(e, d, lambda a, b: EmpFloor(a.name, a.department, b.floor, a.salary))


class SalaryByFloor(AggregateComp):
    def get_key_projection(self, e):
        return make_lambda_from_member(e, "floor")

    def get_value_projection(self, e):
        return make_lambda_from_member(e, "salary")

    def make_output(self, keys, values):
        ks = keys.tolist() if hasattr(keys, "tolist") else list(keys)
        return RecordBatch.from_objects([DepartmentTotal(f"floor{k}", float(v)) for k, v in zip(ks, values.tolist())],
                                        DepartmentTotal)
