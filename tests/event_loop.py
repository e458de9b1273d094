"""Test harness: the shape of FedScale's single-process aggregator event loop (test infrastructure).

``Aggregator`` (named like the reference class, so the mixin treats its methods as the reference's own)
restates only what the device path is driven by, in the reference's own order:
* servicer side (gRPC threads, aggregator.py:177-178): ``CLIENT_EXECUTE_COMPLETION`` queues an upload
  through ``add_event_handler`` (:919-963, :830-840) and answers with ``CLIENT_PING`` (:870-917), which
  pops the executor's next event and serialises ``create_client_task`` / ``get_test_config`` /
  ``model_wrapper.get_weights()`` (:902-903) through ``serialize_response`` (:706-715);
* main thread: ``event_monitor`` (:965-1007) pops the queue in arrival order, ``deserialize_response``
  (:695-704), ``client_completion_handler`` (:454-487: q-FedAvg retention, ``update_lock``,
  ``model_in_update += 1``, ``update_weight_aggregation``) and, once a round's K results are in, the
  round reset (:609, :620-623) plus an UPDATE_MODEL broadcast to every executor.
The device mixin goes in front of it exactly as in production: ``class A(DeviceAggregatorMixin,
Aggregator)``.
"""
from __future__ import annotations

import collections
import pickle
import threading
import time
import types

UPLOAD_MODEL, UPDATE_MODEL, CLIENT_TRAIN, MODEL_TEST, DUMMY = (
    "upload_model", "update_model", "train", "model_test", "dummy_event")  # fedscale/cloud/commons.py


class _Resources:
    def __init__(self):
        self.next_id = 0

    def get_next_task(self, executor_id):
        self.next_id += 1
        return self.next_id


class Aggregator:
    def __init__(self, model_wrapper, args, rounds):
        self.model_wrapper = model_wrapper
        self.args = args
        self.rounds_K = list(rounds)  # tasks_round of each round
        self.round = 0
        self.tasks_round = self.rounds_K[0]
        self.model_in_update = 0
        self.model_weights = []
        self.client_training_results = []
        self.stats_util_accumulator = []
        self.update_lock = threading.Lock()
        self.server_events_queue = collections.deque()
        self.individual_client_events = collections.defaultdict(collections.deque)
        self.resource_manager = _Resources()
        self.processed = []  # arrival order the main loop reduced (client ids)
        self.round_done = []  # per round: (version key, host weights) right after the round

    # ---- servicer threads --------------------------------------------------------------------
    def get_client_conf(self, client_id):
        return {"learning_rate": self.args.learning_rate}

    def create_client_task(self, executor_id):
        next_client_id = self.resource_manager.get_next_task(executor_id)
        train_config = {"client_id": next_client_id, "task_config": self.get_client_conf(next_client_id)}
        return train_config, self.model_wrapper.get_weights()

    def get_test_config(self, client_id):
        return {"client_id": client_id}, self.model_wrapper.get_weights()

    def serialize_response(self, responses):
        return pickle.dumps(responses)

    def deserialize_response(self, responses):
        return pickle.loads(responses)

    def add_event_handler(self, client_id, event, meta, data):
        self.server_events_queue.append((client_id, event, meta, data))

    def CLIENT_PING(self, request, context):
        executor_id, client_id = request.executor_id, request.client_id
        response_data = response_msg = "dummy"
        q = self.individual_client_events[executor_id]
        current_event = DUMMY
        if len(q):
            current_event = q.popleft()
            if current_event == CLIENT_TRAIN:
                response_msg, response_data = self.create_client_task(executor_id)
            elif current_event == MODEL_TEST:
                response_msg, response_data = self.get_test_config(client_id)
            elif current_event == UPDATE_MODEL:
                response_data = self.model_wrapper.get_weights()
        return current_event, self.serialize_response(response_msg), self.serialize_response(response_data)

    def CLIENT_EXECUTE_COMPLETION(self, request, context):
        if request.event == UPLOAD_MODEL:
            self.add_event_handler(request.executor_id, request.event, request.meta_result, request.data_result)
        return self.CLIENT_PING(request, context)

    # ---- main thread -------------------------------------------------------------------------
    def client_completion_handler(self, results):
        if self.args.gradient_policy in ["q-fedavg"]:
            self.client_training_results.append(results)
        self.stats_util_accumulator.append(results["utility"])
        self.update_lock.acquire()
        self.model_in_update += 1
        self.update_weight_aggregation(results)
        self.update_lock.release()

    def round_completion_handler(self, executors):
        self.round_done.append(self.model_wrapper.get_weights())
        self.round += 1
        if self.round < len(self.rounds_K):
            self.tasks_round = self.rounds_K[self.round]
        self.model_in_update = 0
        self.client_training_results = []
        self.stats_util_accumulator = []
        for e in executors:  # broadcast UPDATE_MODEL (dispatch_client_events)
            self.individual_client_events[e].append(UPDATE_MODEL)

    def event_monitor(self, executors, deadline_s: float, on_round=None):
        """Reduce queued uploads until every round is complete (raises TimeoutError at the deadline)."""
        t_end = time.monotonic() + deadline_s
        while self.round < len(self.rounds_K):
            if time.monotonic() > t_end:
                raise TimeoutError(f"event loop: round {self.round}, {self.model_in_update} results in")
            if self.server_events_queue:
                client_id, ev, meta, data = self.server_events_queue.popleft()
                assert ev == UPLOAD_MODEL
                res = self.deserialize_response(data)
                self.processed.append(res["client_id"])
                self.client_completion_handler(res)
                if len(self.stats_util_accumulator) == self.tasks_round:
                    if on_round is not None:
                        on_round(self.round)
                    self.round_completion_handler(executors)
            else:
                time.sleep(0.0005)


def request(executor_id, client_id=0, event=DUMMY, data=None):
    return types.SimpleNamespace(executor_id=executor_id, client_id=client_id, event=event, meta_result=b"",
                                 data_result=data, status=True, msg="")
