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
